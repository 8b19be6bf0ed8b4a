// sin or cos of a float argument for the positional encoding (reference src/models.py:36-44:
// torch.sin / torch.cos of 2^i x), as one branch-free evaluation per lane: lane half 0 wants
// sin(a), half 1 cos(a) = sin(a + pi/2), i.e. the same reduction with the quadrant advanced by one.
//
// Reduction: k = rint(a * 2/pi), r = a - k*pi/2 by a three-constant Cody-Waite split, each step one
// fma (exact product inside, one rounding): |r| <= pi/4 with an absolute error of about 2^-25 for
// |k| < 2^13 (|a| < ~12800).  Polynomials: the Cephes sinf / cosf minimax forms on [-pi/4, pi/4]
// (about 1 ulp).  Measured against double-precision sin/cos over |a| < 8192 by
// tests/test_capi_host.py::test_pe_sin_accuracy (host build of this header).  Arguments beyond
// kPeSinMax take the library sincosf.
#pragma once
#include <math.h>

#if defined(__HIPCC__)
#define NERF_PE_HD __host__ __device__
#else
#define NERF_PE_HD
#endif

namespace nerf {

constexpr float kPeSinMax = 8192.0f;

NERF_PE_HD inline float pe_sin_poly(float r, int q) {
  const float z = r * r;
  float s = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  s = fmaf(s * z, r, r);
  float c = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  c = fmaf(c * z, z, fmaf(-0.5f, z, 1.0f));
  const float v = (q & 1) ? c : s;
  return (q & 2) ? -v : v;
}

// sin(a) for h = 0, cos(a) for h = 1; |a| <= kPeSinMax.
NERF_PE_HD inline float pe_sin_reduced(float a, int h) {
  const float k = rintf(a * 0.636619772367581343f);            // 2/pi
  float r = fmaf(-k, 1.57079637050628662109375f, a);            // float(pi/2)
  r = fmaf(-k, -4.371138828673793e-8f, r);                     // float(pi/2 - c1)
  r = fmaf(-k, -1.7151245100058819e-15f, r);                   // float(pi/2 - c1 - c2)
  return pe_sin_poly(r, (int)k + h);
}

}  // namespace nerf
