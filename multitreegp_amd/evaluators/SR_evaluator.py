"""Import-path mirror of MultiTreeGP/evaluators/SR_evaluator.py."""
from . import SREvaluator as Evaluator  # noqa: F401
from . import RK4, ConstantStepSize  # noqa: F401
