from . import callbacks, loggers  # noqa: F401
