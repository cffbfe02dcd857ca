"""Inert stand-in (see gym/__init__.py)."""
