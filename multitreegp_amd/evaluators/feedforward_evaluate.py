"""Import-path mirror of MultiTreeGP/evaluators/feedforward_evaluate.py."""
from . import FeedforwardEvaluator as Evaluator  # noqa: F401
from . import RK4, ConstantStepSize  # noqa: F401
