// ecnf_part.hip — one compiled shape of the kernels (split build, __graft_entry__.build()): explicit instantiation
// of the launchers of (M, L, D) = (ECNF_PART_M, ECNF_PART_L, ECNF_PART_D), with the tangent kernels when
// ECNF_PART_TAN is 1.
#include "ecnf_kernels.hpp"

namespace ecnf {
ECNF_INST_SHAPE(template, ECNF_PART_M, ECNF_PART_L, ECNF_PART_D, 0)
#if ECNF_PART_TAN
ECNF_INST_SHAPE(template, ECNF_PART_M, ECNF_PART_L, ECNF_PART_D, 1)
#endif
}  // namespace ecnf
