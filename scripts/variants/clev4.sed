# diagnostic variant: the chain kernel's wave-priority levels in quarters of a unit's steps
# (the product: 32nds)
s|const int64_t pstep = ustep >= 64 ? ustep >> 5 : 2;|const int64_t pstep = ustep >= 8 ? ustep >> 2 : 2;|
