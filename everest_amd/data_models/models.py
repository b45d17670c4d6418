"""Kernel, prior, surrogate, acquisition-function and strategy data models on the
GP/qNEHVI path (same names, defaults and ``type`` tags as BoFire):

* kernels  — bofire/data_models/kernels/continuous.py:12-30
* priors   — bofire/data_models/priors/{normal,gamma,api}.py
* surrogate — bofire/data_models/surrogates/single_task_gp.py:106-128,
  trainable_botorch.py:9-30, botorch_surrogates.py
* strategies — bofire/data_models/strategies/predictives/{botorch,qehvi,qnehvi,sobo}.py,
  bofire/data_models/strategies/strategy.py
"""
from __future__ import annotations

import math
from enum import Enum
from typing import Annotated, Dict, List, Literal, Optional, Union

from pydantic import Field, PositiveInt, field_validator, model_validator

from .domain import (BaseModel, CategoricalInput, CloseToTargetObjective, ContinuousOutput, Domain, Inputs,
                     MaximizeObjective, MinimizeObjective, Outputs)


class CategoricalEncodingEnum(str, Enum):
    ORDINAL = "ORDINAL"
    ONE_HOT = "ONE_HOT"
    DUMMY = "DUMMY"
    DESCRIPTOR = "DESCRIPTOR"


class ScalerEnum(str, Enum):
    NORMALIZE = "NORMALIZE"
    STANDARDIZE = "STANDARDIZE"
    IDENTITY = "IDENTITY"


class CategoricalMethodEnum(str, Enum):
    EXHAUSTIVE = "EXHAUSTIVE"
    FREE = "FREE"


def _is_power_of_two(v: int) -> int:
    if v <= 0 or (v & (v - 1)) != 0:
        raise ValueError(f"{v} is not a power of two")
    return v


IntPowerOfTwo = Annotated[int, Field(gt=0)]


# ---------------------------------------------------------------------------------------
# priors
# ---------------------------------------------------------------------------------------
class NormalPrior(BaseModel):
    type: Literal["NormalPrior"] = "NormalPrior"
    loc: float
    scale: Annotated[float, Field(gt=0)]


class LogNormalPrior(BaseModel):
    type: Literal["LogNormalPrior"] = "LogNormalPrior"
    loc: float
    scale: float


class GammaPrior(BaseModel):
    type: Literal["GammaPrior"] = "GammaPrior"
    concentration: Annotated[float, Field(gt=0)]
    rate: Annotated[float, Field(gt=0)]


class DimensionalityScaledLogNormalPrior(BaseModel):
    """Hvarfner et al. prior (bofire/data_models/priors/normal.py:37-49)."""
    type: Literal["DimensionalityScaledLogNormalPrior"] = "DimensionalityScaledLogNormalPrior"
    loc: Annotated[float, Field(gt=0)] = math.sqrt(2)
    loc_scaling: Annotated[float, Field(gt=0)] = 0.5
    scale: Annotated[float, Field(gt=0)] = math.sqrt(3)
    scale_scaling: float = 0.0


AnyPrior = Annotated[Union[NormalPrior, LogNormalPrior, GammaPrior, DimensionalityScaledLogNormalPrior],
                     Field(discriminator="type")]


def HVARFNER_NOISE_PRIOR():  # bofire/data_models/priors/api.py:50
    return LogNormalPrior(loc=-4, scale=1)


def HVARFNER_LENGTHSCALE_PRIOR():
    return DimensionalityScaledLogNormalPrior()


# ---------------------------------------------------------------------------------------
# kernels
# ---------------------------------------------------------------------------------------
class RBFKernel(BaseModel):
    type: Literal["RBFKernel"] = "RBFKernel"
    features: Optional[List[str]] = None
    ard: bool = True
    lengthscale_prior: Optional[AnyPrior] = None


class MaternKernel(BaseModel):
    type: Literal["MaternKernel"] = "MaternKernel"
    features: Optional[List[str]] = None
    ard: bool = True
    nu: float = 2.5
    lengthscale_prior: Optional[AnyPrior] = None

    @field_validator("nu")
    @classmethod
    def _nu(cls, nu):
        if nu not in {0.5, 1.5, 2.5}:
            raise ValueError("nu expected to be 0.5, 1.5, or 2.5")
        return nu


AnyKernel = Annotated[Union[RBFKernel, MaternKernel], Field(discriminator="type")]


# ---------------------------------------------------------------------------------------
# surrogates
# ---------------------------------------------------------------------------------------
class SingleTaskGPSurrogate(BaseModel):
    type: Literal["SingleTaskGPSurrogate"] = "SingleTaskGPSurrogate"
    inputs: Inputs
    outputs: Outputs
    input_preprocessing_specs: Dict[str, CategoricalEncodingEnum] = Field(default_factory=dict, validate_default=True)
    dump: Optional[str] = None
    scaler: ScalerEnum = ScalerEnum.NORMALIZE
    output_scaler: ScalerEnum = ScalerEnum.STANDARDIZE
    kernel: AnyKernel = Field(default_factory=lambda: RBFKernel(ard=True,
                                                                lengthscale_prior=HVARFNER_LENGTHSCALE_PRIOR()))
    noise_prior: AnyPrior = Field(default_factory=HVARFNER_NOISE_PRIOR)

    @field_validator("output_scaler")
    @classmethod
    def _os(cls, v):
        if v == ScalerEnum.NORMALIZE:
            raise ValueError("Normalize is not supported as an output transform.")
        return v

    @model_validator(mode="after")
    def _specs(self):
        """Botorch models one-hot encode categoricals (bofire/data_models/surrogates/botorch.py:19-60)."""
        specs = dict(self.input_preprocessing_specs)
        for key in self.inputs.get_keys(CategoricalInput):
            if specs.get(key, CategoricalEncodingEnum.ONE_HOT) != CategoricalEncodingEnum.ONE_HOT:
                raise ValueError("Botorch based models have to use one hot encodings for categoricals")
            specs[key] = CategoricalEncodingEnum.ONE_HOT
        self.__dict__["input_preprocessing_specs"] = specs
        if len(self.outputs) != 1:
            raise ValueError("SingleTaskGPSurrogate takes exactly one output")
        return self


AnySurrogate = Annotated[Union[SingleTaskGPSurrogate], Field(discriminator="type")]


class BotorchSurrogates(BaseModel):
    type: Literal["BotorchSurrogates"] = "BotorchSurrogates"
    surrogates: List[AnySurrogate] = Field(default_factory=list)

    @property
    def input_preprocessing_specs(self):
        specs = {}
        for s in self.surrogates:
            specs.update(s.input_preprocessing_specs)
        return specs

    @property
    def outputs(self) -> Outputs:
        feats = []
        for s in self.surrogates:
            feats += list(s.outputs.features)
        return Outputs(features=feats)


# ---------------------------------------------------------------------------------------
# acquisition functions (bofire/data_models/acquisition_functions/acquisition_function.py)
# ---------------------------------------------------------------------------------------
class _AcqfMC(BaseModel):
    """n_mc_samples must be a power of two (bofire IntPowerOfTwo)."""

    @field_validator("n_mc_samples", check_fields=False)
    @classmethod
    def _p2mc(cls, v):
        return _is_power_of_two(v)


class qEI(_AcqfMC):
    type: Literal["qEI"] = "qEI"
    n_mc_samples: int = 512


class qLogEI(_AcqfMC):
    type: Literal["qLogEI"] = "qLogEI"
    n_mc_samples: int = 512


class qNEI(_AcqfMC):
    type: Literal["qNEI"] = "qNEI"
    prune_baseline: bool = True
    n_mc_samples: int = 512


class qLogNEI(_AcqfMC):
    type: Literal["qLogNEI"] = "qLogNEI"
    prune_baseline: bool = True
    n_mc_samples: int = 512


class qEHVI(_AcqfMC):
    type: Literal["qEHVI"] = "qEHVI"
    alpha: Annotated[float, Field(ge=0)] = 0.0
    n_mc_samples: int = 512


class qLogEHVI(_AcqfMC):
    type: Literal["qLogEHVI"] = "qLogEHVI"
    alpha: Annotated[float, Field(ge=0)] = 0.0
    n_mc_samples: int = 512


class qNEHVI(_AcqfMC):
    type: Literal["qNEHVI"] = "qNEHVI"
    alpha: Annotated[float, Field(ge=0)] = 0.0
    prune_baseline: bool = True
    n_mc_samples: int = 512


class qLogNEHVI(_AcqfMC):
    type: Literal["qLogNEHVI"] = "qLogNEHVI"
    alpha: Annotated[float, Field(ge=0)] = 0.0
    prune_baseline: bool = True
    n_mc_samples: int = 512


AnyMultiObjectiveAcquisitionFunction = Annotated[Union[qEHVI, qLogEHVI, qNEHVI, qLogNEHVI],
                                                 Field(discriminator="type")]
AnySingleObjectiveAcquisitionFunction = Annotated[Union[qEI, qLogEI, qNEI, qLogNEI], Field(discriminator="type")]


# ---------------------------------------------------------------------------------------
# strategies
# ---------------------------------------------------------------------------------------
class Strategy(BaseModel):
    type: str
    domain: Domain
    seed: Optional[Annotated[int, Field(ge=0)]] = None


class RandomStrategy(Strategy):
    type: Literal["RandomStrategy"] = "RandomStrategy"


class BotorchStrategy(Strategy):
    """bofire/data_models/strategies/predictives/botorch.py:77-253 (the fields on this path)."""
    num_restarts: PositiveInt = 8
    num_raw_samples: IntPowerOfTwo = 1024
    maxiter: PositiveInt = 2000
    batch_limit: Optional[PositiveInt] = Field(default=None, validate_default=True)
    descriptor_method: CategoricalMethodEnum = CategoricalMethodEnum.EXHAUSTIVE
    categorical_method: CategoricalMethodEnum = CategoricalMethodEnum.EXHAUSTIVE
    discrete_method: CategoricalMethodEnum = CategoricalMethodEnum.EXHAUSTIVE
    surrogate_specs: BotorchSurrogates = Field(default_factory=BotorchSurrogates, validate_default=True)
    frequency_hyperopt: Annotated[int, Field(ge=0)] = 0
    folds: int = 5

    @field_validator("num_raw_samples")
    @classmethod
    def _p2(cls, v):
        return _is_power_of_two(v)

    @field_validator("batch_limit")
    @classmethod
    def _bl(cls, batch_limit, info):
        return min(batch_limit or info.data["num_restarts"], info.data["num_restarts"])

    @model_validator(mode="after")
    def _surrogates(self):
        """_generate_surrogate_specs: one default SingleTaskGPSurrogate per output without a
        spec (bofire/data_models/strategies/predictives/botorch.py:195-239).  The reference
        picks MixedSingleTaskGP when categorical inputs exist — out of scope here; such
        domains need explicit SingleTaskGPSurrogate specs (one-hot inputs)."""
        specs = self.surrogate_specs
        have = set(specs.outputs.get_keys())
        new = list(specs.surrogates)
        for key in sorted(set(self.domain.outputs.get_keys()) - have):
            if len(self.domain.inputs.get(CategoricalInput, exact=True).features):
                raise ValueError(f"output `{key}`: categorical inputs need an explicit SingleTaskGPSurrogate spec "
                                 "(MixedSingleTaskGP is out of scope for the MI355X build)")
            new.append(SingleTaskGPSurrogate(inputs=self.domain.inputs,
                                             outputs=Outputs(features=[self.domain.outputs.get_by_key(key)])))
        specs.__dict__["surrogates"] = new
        for s in new:
            for k in s.outputs.get_keys():
                if k not in self.domain.outputs.get_keys():
                    raise KeyError(f"surrogate output `{k}` not in domain")
        return self


_MO_CONSTRAINED = ("MaximizeObjective", "MinimizeObjective", "MinimizeSigmoidObjective", "MaximizeSigmoidObjective",
                   "TargetObjective", "CloseToTargetObjective")


def _check_objectives(cls, domain: Domain, allowed) -> Domain:
    """bofire/data_models/strategies/strategy.py:26-34 (is_objective_implemented)."""
    for f in domain.outputs.get().features:
        obj = getattr(f, "objective", None)
        if obj is not None and type(obj).__name__ not in allowed:
            raise ValueError(f"Objective `{type(obj)}` is not implemented for strategy `{cls.__name__}`")
    return domain


class MultiobjectiveStrategy(BotorchStrategy):
    @field_validator("domain")
    @classmethod
    def _mo(cls, v):
        feats = v.outputs.get_by_objective([MaximizeObjective, MinimizeObjective, CloseToTargetObjective])
        if len(feats) < 2:
            raise ValueError("At least two output features with MaximizeObjective or MinimizeObjective has to be "
                             "defined in the domain.")
        for f in feats.features:
            if f.objective.w != 1.0:
                raise ValueError(f"Only objectives with weight 1 are supported. Violated by feature {f.key}.")
        return v


class QehviStrategy(MultiobjectiveStrategy):
    type: Literal["QehviStrategy"] = "QehviStrategy"
    num_sobol_samples: IntPowerOfTwo = 512
    ref_point: Optional[Dict[str, float]] = None

    @field_validator("domain")
    @classmethod
    def _objectives(cls, v):
        """bofire/data_models/strategies/predictives/qehvi.py:53-67."""
        return _check_objectives(cls, v, ("MaximizeObjective", "MinimizeObjective"))

    @field_validator("num_sobol_samples")
    @classmethod
    def _p2s(cls, v):
        return _is_power_of_two(v)

    @model_validator(mode="after")
    def _ref(self):
        if self.ref_point is None:
            return self
        keys = self.domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective,
                                                          CloseToTargetObjective])
        if sorted(keys) != sorted(self.ref_point.keys()):
            raise ValueError(f"Provided refpoint do not match the domain, expected keys: {keys}")
        return self


class QnehviStrategy(QehviStrategy):
    type: Literal["QnehviStrategy"] = "QnehviStrategy"
    alpha: Annotated[float, Field(ge=0, le=0.5)] = 0.0

    @field_validator("domain")
    @classmethod
    def _objectives(cls, v):
        """bofire/data_models/strategies/predictives/qnehvi.py:21-39."""
        return _check_objectives(cls, v, _MO_CONSTRAINED)


class MoboStrategy(MultiobjectiveStrategy):
    """bofire/data_models/strategies/predictives/mobo.py:24-80."""
    type: Literal["MoboStrategy"] = "MoboStrategy"
    ref_point: Optional[Dict[str, float]] = None
    acquisition_function: AnyMultiObjectiveAcquisitionFunction = Field(default_factory=qLogNEHVI)

    @field_validator("domain")
    @classmethod
    def _objectives(cls, v):
        """bofire/data_models/strategies/predictives/mobo.py:60-80."""
        return _check_objectives(cls, v, _MO_CONSTRAINED)

    @model_validator(mode="after")
    def _ref(self):
        if self.ref_point is None:
            return self
        keys = self.domain.outputs.get_keys_by_objective([MaximizeObjective, MinimizeObjective,
                                                          CloseToTargetObjective])
        if sorted(keys) != sorted(self.ref_point.keys()):
            raise ValueError(f"Provided refpoint do not match the domain, expected keys: {keys}")
        return self


class SoboStrategy(BotorchStrategy):
    type: Literal["SoboStrategy"] = "SoboStrategy"
    acquisition_function: AnySingleObjectiveAcquisitionFunction = Field(default_factory=qLogNEI)


AnyStrategy = Annotated[Union[QnehviStrategy, QehviStrategy, MoboStrategy, SoboStrategy, RandomStrategy],
                       Field(discriminator="type")]
