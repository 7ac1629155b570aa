"""tools subpackage."""
