# diagnostic variant: the grid kernel's wave-priority levels in 128ths of a unit's steps
# (the product: 32nds)
s|const uint32_t pstep = ustep >= 64u ? ustep >> 5 : 2u;|const uint32_t pstep = ustep >= 256u ? ustep >> 7 : 2u;|
