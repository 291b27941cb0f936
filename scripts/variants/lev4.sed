# diagnostic variant: the grid kernel's wave-priority levels in 4ths of a unit's steps
s|const uint32_t pstep = ustep >= 64u ? ustep >> 5 : 2u;|const uint32_t pstep = ustep >= 8u ? ustep >> 2 : 2u;|
