// The grid kernel's W2 instantiations (fw_grid16.hip: the lean R = 1 kernel without the
// 3-wave register budget, for launches with at most 2 waves of work per SIMD -- the 8-GPU
// job's 8,192-chain shards) in a translation unit of their own, so the Makefile schedules
// them with LLVM's max-ILP strategy (Makefile).
// The stamps build compiles them in fw_grid16.hip instead.
#ifndef FW_STAMPS
#define FW_G16_W2_TU 1
#include "fw_grid16.hip"
#endif
