"""Dependency-free helpers (block layout, logging, metrics, timers)."""
