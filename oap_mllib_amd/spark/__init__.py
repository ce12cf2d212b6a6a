"""spark subpackage."""
