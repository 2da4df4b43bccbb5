"""Inference math: reference-compatible API and the float64 oracle."""
from ..utils.blocks import (LazyBlockDiag, blocks_to_sparse, interleaved_to_soa, ntri, pack_blocks,  # noqa: F401
                     pack_matrix, soa_to_interleaved, sparse_to_blocks, tri_indices, tri_pos, unpack_blocks,
                     unpack_matrix)
from .kf_tools import (NoHessianMethod, PropagatorSpec, blend_prior, hessian_correction,  # noqa: F401
                       hessian_correction_multiband, hessian_correction_pixel, identity_propagation,
                       make_no_propagation, make_partial_prior_propagator, no_propagation,
                       propagate_and_blend_prior, propagate_information_filter, propagate_information_filter_approx_SLOW,
                       propagate_information_filter_LAI, propagate_information_filter_SLOW, propagate_standard_kalman,
                       tip_prior_full, tip_prior_noLAI)
from .solvers import (analysis_blocks, gain_blocks, sort_band_data, variational_kalman,  # noqa: F401
                      variational_kalman_multiband)
from .utils import (block_diag, create_linear_observation_operator, create_nonlinear_observation_operator,  # noqa
                    create_prosail_observation_operator, create_sar_observation_operator, create_uncertainty,
                    iterate_time_grid, locate_in_lut, run_emulator, spsolve2)
from ..models.priors import tip_prior  # noqa: F401
from ..models.operators import band_selecta  # noqa: F401
