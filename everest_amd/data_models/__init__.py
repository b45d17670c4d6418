from .domain import (BaseModel, CategoricalInput, CloseToTargetObjective, ConstrainedObjective, Constraints, ConstraintNotFulfilledError,
                     ContinuousInput, ContinuousOutput, Domain, Inputs, LinearEqualityConstraint,
                     LinearInequalityConstraint, MaximizeObjective, MaximizeSigmoidObjective, MinimizeObjective,
                     MinimizeSigmoidObjective, MovingMaximizeSigmoidObjective, Outputs, TargetObjective)
from .models import (BotorchSurrogates, CategoricalEncodingEnum, CategoricalMethodEnum,
                     DimensionalityScaledLogNormalPrior, GammaPrior, LogNormalPrior, MaternKernel, NormalPrior,
                     QehviStrategy, QnehviStrategy, RandomStrategy, RBFKernel, ScalerEnum, SingleTaskGPSurrogate,
                     SoboStrategy, MoboStrategy, qEHVI, qEI, qLogEHVI, qLogEI, qLogNEHVI, qLogNEI, qNEHVI,
                     qNEI)
