// Tile / group bounding boxes of the prefilter records and the box test the
// tile-pair cull (K0d, bsa_cd.hip) and the halo plan of the row-sharded step
// (bsa_halo.hip) share: both must take the same decision for the same boxes.
#pragma once
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

__device__ __forceinline__ TileBox box_union(const TileBox &a, const TileBox &b) {
  TileBox u;
  for (int q = 0; q < 3; ++q) {
    u.lo[q] = fminf(a.lo[q], b.lo[q]);
    u.hi[q] = fmaxf(a.hi[q], b.hi[q]);
  }
  u.vlo = fminf(a.vlo, b.vlo);
  u.vhi = fmaxf(a.vhi, b.vhi);
  u.smax = fmaxf(a.smax, b.smax);
  u.pad0 = 0.f;
  u.count = a.count + b.count;
  u.pad1 = 0;
  return u;
}

__device__ __forceinline__ float gap(float alo, float ahi, float blo, float bhi) {
  return fmaxf(0.f, fmaxf(alo - bhi, blo - ahi));
}

// Can any pair of the two boxes pass stage 1?  Horizontally the gaps bound the
// chord from below and s_i + s_j <= smax_a + smax_b; vertically stage 1 needs
// lo_j < hi_i and hi_j > lo_i, so the [vlo, vhi] intervals must overlap.
// Symmetric, bitwise: swapping a and b swaps the operands of fmaxf, of the
// smax sum and of the two comparisons only (no contraction, -ffp-contract=off),
// so the sender and the receiver of a halo tile take the same decision.
__device__ __forceinline__ bool boxes_may_interact(const TileBox &a, const TileBox &b) {
  const float gx = gap(a.lo[0], a.hi[0], b.lo[0], b.hi[0]);
  const float gy = gap(a.lo[1], a.hi[1], b.lo[1], b.hi[1]);
  const float gz = gap(a.lo[2], a.hi[2], b.lo[2], b.hi[2]);
  const float d2 = gx * gx + gy * gy + gz * gz;
  const float st = (a.smax + b.smax) * 1.00001f + 1e-5f;
  return !(d2 >= st * st) && (b.vlo < a.vhi) && (b.vhi > a.vlo);
}

// Tile-pair list reuse: a box grown by dx in every unit-vector
// axis, ds in reach and dv vertically (plus a rounding margin far above one
// fp32 ulp of the values), and the matching per-record test -- a record within
// (dx, ds, dv) of its record at the build lies inside every box grown from a
// box that held the build record, so every pair the boxes of the current
// records could keep, the grown boxes of the build kept (boxes_may_interact is
// monotone in the extents).  NaN fails the test (a rebuild), never passes it.
constexpr float kTprPad = 1e-6f;   // chord / reach units (fp32 ulp of a unit vector ~6e-8)
constexpr float kTprPadV = 1.0f;   // m (fp32 ulp at 20 km ~2e-3)
__device__ __forceinline__ TileBox box_grow(TileBox b, float dx, float ds, float dv) {
  for (int q = 0; q < 3; ++q) {
    b.lo[q] -= dx + kTprPad;
    b.hi[q] += dx + kTprPad;
  }
  b.smax += ds + kTprPad;
  b.vlo -= dv + kTprPadV;
  b.vhi += dv + kTprPadV;
  return b;
}
__device__ __forceinline__ bool pf_within(const PFRec &p, const PFRec &b, float dx, float ds, float dv) {
  return fabsf(p.x - b.x) <= dx && fabsf(p.y - b.y) <= dx && fabsf(p.z - b.z) <= dx && p.s <= b.s + ds &&
         p.lo >= b.lo - dv && p.hi <= b.hi + dv;
}

}  // namespace bsa
