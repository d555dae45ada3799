"""Minimal stand-in for python-future (fixture generation only)."""
