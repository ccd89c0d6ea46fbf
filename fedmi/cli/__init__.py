"""Command-line entry points (server / client / standalone train)."""
