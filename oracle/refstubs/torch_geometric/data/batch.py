from . import Batch  # noqa: F401
