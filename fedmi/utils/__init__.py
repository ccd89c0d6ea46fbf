"""Checkpoint-independent helpers."""
