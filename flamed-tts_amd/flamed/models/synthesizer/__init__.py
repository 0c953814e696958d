from .prob_generator import ProbGenerator  # noqa: F401


def __getattr__(name):
    if name == "PriorGenerator":
        from .prior_generator import PriorGenerator
        return PriorGenerator
    if name == "PVA":
        from .pva import PVA
        return PVA
    raise AttributeError(name)
