"""Inert stand-in (see gym/__init__.py): records ids only."""
registry = {}


def register(id, entry_point=None, **kwargs):
    registry[id] = entry_point
