class Callback:
    pass


class BatchSizeFinder:
    def __init__(self, *a, **k):
        pass
