# diagnostic variant: the grid kernel's wave-priority levels in 8ths of a unit's steps
s|const uint32_t pstep = ustep >= 64u ? ustep >> 5 : 2u;|const uint32_t pstep = ustep >= 16u ? ustep >> 3 : 2u;|
