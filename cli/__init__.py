"""Drop-in alias of the reference's `cli` package (src/cli/)."""
