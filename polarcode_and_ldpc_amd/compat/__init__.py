"""Import shim reproducing the reference's `src/` layout (see README.md here)."""
