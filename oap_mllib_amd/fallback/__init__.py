"""fallback subpackage."""
