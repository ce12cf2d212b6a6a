"""persistence subpackage."""
