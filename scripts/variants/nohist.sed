# diagnostic variant (not a product build): every yield-histogram flush dropped, so a PMC
# pass sizes the histogram atomics' share of WRITE_SIZE (grid kernel and chain kernel)
s|^#define HIST_ADD(ptr, v) atomicAdd(ptr, v)|#define HIST_ADD(ptr, v) ((void)(ptr), (void)(v))|
s|if (hc) atomicAdd(p.hist_cut + base_c + lane, (unsigned long long)hc);|(void)hc;|
s|if (hb) atomicAdd(p.hist_b + base_b + lane, (unsigned long long)hb);|(void)hb;|
