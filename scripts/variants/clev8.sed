# diagnostic variant: the chain kernel's wave-priority levels in 8ths of a unit's steps
s|const int64_t pstep = ustep >= 64 ? ustep >> 5 : 2;|const int64_t pstep = ustep >= 16 ? ustep >> 3 : 2;|
