"""Import-path mirror of MultiTreeGP/evaluators/dynamic_evaluate.py."""
from . import DynamicEvaluator as Evaluator  # noqa: F401
from . import RK4, ConstantStepSize  # noqa: F401
