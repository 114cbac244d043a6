"""sim subpackage."""
