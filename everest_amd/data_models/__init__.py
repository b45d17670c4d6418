from .domain import (BaseModel, CategoricalInput, CloseToTargetObjective, Constraints, ConstraintNotFulfilledError,
                     ContinuousInput, ContinuousOutput, Domain, Inputs, LinearEqualityConstraint,
                     LinearInequalityConstraint, MaximizeObjective, MinimizeObjective, Outputs)
from .models import (BotorchSurrogates, CategoricalEncodingEnum, CategoricalMethodEnum,
                     DimensionalityScaledLogNormalPrior, GammaPrior, LogNormalPrior, MaternKernel, NormalPrior,
                     QehviStrategy, QnehviStrategy, RandomStrategy, RBFKernel, ScalerEnum, SingleTaskGPSurrogate,
                     SoboStrategy, MoboStrategy, qEHVI, qEI, qLogEHVI, qLogEI, qLogNEHVI, qLogNEI, qNEHVI,
                     qNEI)
