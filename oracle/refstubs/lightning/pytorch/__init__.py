from . import callbacks  # noqa: F401
