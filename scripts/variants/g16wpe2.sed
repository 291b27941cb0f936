# diagnostic variant: the grid kernel (R = 1) under a 2-waves-per-SIMD register budget
# (up to 256 VGPRs): does a larger budget shorten a wave's iteration where only 2 waves
# per SIMD have work (the 8,192-chain shard)?
s|__global__ __launch_bounds__(64 \* MAX_NW) void fw_grid16_kernel(FwRunParams p) {|__global__ __launch_bounds__(64 * MAX_NW) __attribute__((amdgpu_waves_per_eu(2, 2))) void fw_grid16_kernel(FwRunParams p) {|
