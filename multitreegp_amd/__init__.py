"""multitreegp_amd -- MI355X-native population-fitness evaluator for MultiTreeGP.

Hot path: GeneticProgramming.evaluate_population and the evaluators/
fitness plugins, rebuilt as a tree->program flattener plus one fused HIP kernel that
interprets the programs inside a fixed-step RK4 integrator (multitreegp_amd/csrc).
"""
from .node_library import NodeLibrary  # noqa: F401
from .environments import Acrobot, HarmonicOscillator, StirredTankReactor, VanDerPolOscillator, LinearSystem, control_data, ground_truth  # noqa: F401
from .evaluators import (RK4, Euler, ConstantStepSize, Dopri5, PIDController, DynamicEvaluator, FeedforwardEvaluator,  # noqa: F401
                         SREvaluator)
from .genetic_programming import GeneticProgramming, TreeEvaluator  # noqa: F401

__version__ = "0.1.0"
