def __getattr__(name):
    if name == "Flamed":
        from .flamed import Flamed
        return Flamed
    raise AttributeError(name)
