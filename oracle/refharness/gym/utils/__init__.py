"""Inert stand-in (see gym/__init__.py)."""
from . import seeding  # noqa: F401
