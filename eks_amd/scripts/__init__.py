"""Command-line entry points mirroring the reference scripts/ (F1)."""
