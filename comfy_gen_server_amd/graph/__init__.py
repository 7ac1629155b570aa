"""graph subpackage."""
