"""sampling subpackage."""
