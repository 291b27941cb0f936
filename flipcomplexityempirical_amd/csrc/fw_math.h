// fw_math.h — fp64 helpers evaluated identically on the host and on gfx950.
//
// The sampled geometric waits (fw_chains_enable_waits, include/flipwalk.h) must be bit
// for bit the C oracle's (oracle/flipchain_oracle.c: orc_log1p, wait_draw), so log1p is
// spelled out here in IEEE double operations the compiler may neither fuse nor reorder,
// instead of calling the device or host libm (which differ in the last bit).
#pragma once

#include <stdint.h>
#include <string.h>

#include <hip/hip_runtime.h>

// log1p(x) for -1 < x <= 0: 1 + x = 2^k m with m in [sqrt(2)/2, sqrt(2)); log m =
// 2 atanh(f / (2 + f)), f = m - 1, by a degree-14 odd series; plus the rounding correction
// of 1 + x.  The same operation sequence as orc_log1p.
__host__ __device__ inline double fw_log1p(double x) {
#pragma clang fp contract(off)
  if (x == 0.0) return x;
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  const double u = 1.0 + x;
  uint64_t bits;
  memcpy(&bits, &u, 8);
  int k = (int)((bits >> 52) & 0x7FF) - 1023;
  uint64_t mb = (bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull;
  if (mb > 0x3FF6A09E667F3BCCull) {  // m >= sqrt(2): halve it
    mb -= 0x0010000000000000ull;
    k += 1;
  }
  double m;
  memcpy(&m, &mb, 8);
  double c = k > 0 ? 1.0 - (u - x) : x - (u - 1.0);
  c = c / u;
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + (dk * ln2_lo + c))) - f);
}

// attempt index of the initial state's wait draw (no proposal attempt creates it)
#define FW_WAIT_T0 0x7FFFFFFFFFFFFFFFull
