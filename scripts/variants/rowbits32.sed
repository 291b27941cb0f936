# experiment: a row's 16 ballot bits by a 32-bit select + bfe instead of a 64-bit shift
s|^  return (uint32_t)(bal >> (row \* ROW)) \& 0xFFFFu;|  const uint32_t h_ = (row \& 2) ? (uint32_t)(bal >> 32) : (uint32_t)bal; return __builtin_amdgcn_ubfe(h_, (uint32_t)(row \& 1) << 4, 16);|
