// The grid kernel's small-grid lean instantiations (fw_grid16.hip: R = 1, at most 256 weight
// groups, cut_accept, no optional features -- C3 and its 2- and 4-GPU shards) in a
// translation unit of their own, so the Makefile schedules them with LLVM's iterative-ILP
// strategy; the speculative, large-grid and FULL ones keep the default schedule (no
// scratch: the ILP strategies spill them).  The stamps build compiles them in
// fw_grid16.hip instead.
#ifndef FW_STAMPS
#define FW_G16_LEAN_TU 1
#include "fw_grid16.hip"
#endif
