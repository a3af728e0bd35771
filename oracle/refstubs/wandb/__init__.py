class Config(dict):
    pass
