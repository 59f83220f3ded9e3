"""Command-line front ends (reference: src/cli/)."""
