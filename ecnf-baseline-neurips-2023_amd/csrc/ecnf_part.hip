// ecnf_part.hip — one compiled shape of the kernels (split build, __graft_entry__.build()): explicit instantiation
// of the launchers of (M, L, D) = (ECNF_PART_M, ECNF_PART_L, ECNF_PART_D), with the tangent kernels when
// ECNF_PART_TAN is 1, in the GEMM arithmetic ECNF_PART_PREC (0: split fp16, 1: strict fp32; Geo in egnn_eval.hpp).
// __graft_entry__.build() passes TAN = 1 for every shape (ECNF_SHAPES and ECNF_SHAPES_WIDE_TAN) at both precisions.
#include "ecnf_kernels.hpp"

namespace ecnf {
ECNF_INST_SHAPE(template, ECNF_PART_M, ECNF_PART_L, ECNF_PART_D, 0, ECNF_PART_PREC)
#if ECNF_PART_TAN
ECNF_INST_SHAPE(template, ECNF_PART_M, ECNF_PART_L, ECNF_PART_D, 1, ECNF_PART_PREC)
#endif
}  // namespace ecnf
