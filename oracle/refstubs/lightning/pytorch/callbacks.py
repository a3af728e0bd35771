class Callback:
    pass


class BatchSizeFinder:
    def __init__(self, *a, **k):
        pass


class EarlyStopping(Callback):  # import-only stand-in
    def __init__(self, *a, **k):
        pass


class ModelCheckpoint(Callback):  # import-only stand-in
    def __init__(self, *a, **k):
        pass
