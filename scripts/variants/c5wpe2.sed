# diagnostic variant: the 3-bit grid chain kernel (C5) under a 2-waves-per-SIMD register
# budget (256 VGPRs, no spills; 8 chains per CU instead of 10)
s|pick_per<3, true, 2, false, 3, FULL>(G) : pick_per<3, true, 1, false, 3, FULL>(G)|pick_per<3, true, 2, false, 2, FULL>(G) : pick_per<3, true, 1, false, 2, FULL>(G)|
