"""nodes subpackage."""
