"""Utilities: timers/profiler, logging, parameters."""
