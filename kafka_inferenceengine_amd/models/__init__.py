"""Model families: priors, GP emulators (PROSAIL / JRC-TIP), SAR Water Cloud Model, operators."""
from .gp import GaussianProcessEmulator, make_prosail_emulators, make_tip_emulators  # noqa: F401
from .operators import (OP_GP, OP_LINEAR, OP_PRECOMP, OP_SAR, TIP_BAND_MAPPER, LinearOperator,  # noqa: F401
                        OperatorSpec, band_selecta, create_linear_observation_operator,
                        create_nonlinear_observation_operator, create_prosail_observation_operator,
                        create_sar_observation_operator, gp_spec)
from .priors import (SAIL_PARAMETERS, TIP_PARAMETERS, DevicePrior, GaussianPrior, JRCPrior,  # noqa: F401
                     SAILPrior, sail_prior, tip_prior)
from .sar import WaterCloudModel, sar_observation_operator  # noqa: F401
