from . import graph_creation  # noqa: F401
