"""Utilities: metrics, timers, health reports, fault injection."""
