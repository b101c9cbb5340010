// K0b / K0c pieces shared by the detect (bsa_cd.hip: k_prep_cols, k_boxes)
// and the resident step's K4' (bsa_sim.hip), which prepares the next CD
// step's column records and boxes from the state it has just computed
// (DESIGN.md 3.7): the same expressions, so the records are bitwise those
// k_prep_cols would write.
#pragma once

#include "bsa_box.h"
#include "bsa_geo_math.h"
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

// Bounds of every group of kGroup (= one wave's 64 lanes) consecutive sorted
// records and of every tile (kTile / kGroup groups).  NaN coordinates drop out
// of the min/max (fminf/fmaxf), which is safe: a record with a NaN coordinate
// never passes the reach test.
constexpr int kGroup = 64;
static_assert(kTile % kGroup == 0, "tiles are whole groups");
constexpr int kGroupsPerTile = kTile / kGroup;
constexpr int kSub = 8;  // column sub-group (culling granularity; one stage-1 chunk)
static_assert(kGroup % kSub == 0 && (kSub & (kSub - 1)) == 0, "sub-groups tile a group");


// ------------------------------------------------------------------ K0b prep
// Horizontal half-bound in unit-sphere chord units: a pair is
// kept iff chord < s_i + s_j,  s = ((R/2 + (|gs| + 0.5e-3) tla)(1 + 1e-5)) / 6.3e6 + 1e-6.
// s >= 0.5 (a reach beyond ~3000 km) or non-finite -> INF (never pruned
// horizontally); the bound also caps the magnitudes in the fp32 test (kPlaneMargin).
__device__ __forceinline__ float reach_h(double rpz, double gs, double tlap) {
  const double s = ((0.5 * rpz + (fabs(gs) + 0.5e-3) * tlap) * (1.0 + 1e-5)) * (1.0 / 6.3e6) + 1e-6;
  return (s < 0.5) ? (float)s : INFINITY;
}
// vertical half-bound [m]: kept iff |dalt| < h_i + h_j
__device__ __forceinline__ double reach_v(double hpz, double vs, double alt, double tlap) {
  return (0.5 * hpz + (fabs(vs) + 0.5e-6) * tlap) * (1.0 + 1e-5) + 0.5 + 1e-6 * fabs(alt);
}

// (Divisions by the constant radii are products with their reciprocals: one
// more rounding, 2^-53 relative, inside the 1e-5 relative and 1e-6 chord
// margins of every bound below; a quarter-rate fp64 division chain fewer each.)
// Prefilter record from the fp64 unit vector, reach and altitude.
// lo / hi = alt -/+ h rounded to fp32 (error
// <= 1e-3 m at flight levels, inside h's 0.5 m + 1e-6 |alt| margin); a
// non-finite h keeps the pair vertically (lo = -INF, hi = +INF).
__device__ __forceinline__ PFRec make_pf(double px, double py, double pz, float s, double alt, double h,
                                         float sv = 0.f) {
  PFRec p;
  p.x = (float)px;
  p.y = (float)py;
  p.z = (float)pz;
  p.s = s;
  if (isfinite(h)) {
    p.lo = (float)(alt - h);
    p.hi = (float)(alt + h);
  } else {
    p.lo = -INFINITY;
    p.hi = INFINITY;
  }
  p.alt = (float)alt;
  p.pad = sv;  // vertical budget of a reusable list (0 otherwise), read by the refine
  return p;
}

// Midpoint stage 1.  A conflict or LoS of a pair needs a
// t* in [0, T] (T = max(tla, 0)) with |D + dV t*| <= R and |dalt + dvs t*| <= H
// in the reference's flat frame at the row (D: its dx / dy, dV: du / dv;
// also when dv2 / dvs were clamped, see 3.2).  Hence |D + dV T/2| <= R + |dV| T/2
// and |dalt + dvs T/2| <= H + |dvs| T/2: every aircraft is tested at its
// position half-way through the look-ahead, m = p + (T/2) (u e + v n) / R_S
// (e, n its own east / north unit vectors), with half the speed reach.  In
// the row's tangent frame m_j - m_i = B_i (p_est + dV T/2) / R_S
// + (T/2) (B_j - B_i) V_j / R_S - (1 - cos c) p_i, where p_est is the chord's
// tangent part (the reference's D = sigma p_est, |1 - sigma| < 0.012 for the
// chords involved), ||B_j - B_i|| <= chord (pi/2 + (1 + pi/2) / rho'), and
// 1 - cos c = chord^2 / 2.  A conflicting pair has chord <= cmax (its dist is
// <= R + (|V_i| + |V_j|) T with every |V| <= kVcap), so
//   s = [(R/2 + |V| T/2)(1 + 1e-5) + 0.012 (R/2 + |V| T) + |V| (T/2) kb cmax] / 6.3e6
//       + cmax^2 / 4 + 1e-6
// per aircraft bounds |m_j - m_i| / 2 for every such pair.  Aircraft faster
// than kVcap, with a non-finite velocity, or within cmax of a pole-ish
// latitude (rho' = cos(lat) - cmax < 0.05) get s = INF (never pruned
// horizontally).  Vertically a = alt + vs T/2, h = H/2 + (|vs| + 1.5e-6) T/2
// (+ the same rounding margins as reach_v; 1.5e-6 covers the dvs clamp).
constexpr double kVcap = 400.0;  // [m/s]
__device__ __forceinline__ PFRec make_pf_mid(double px, double py, double pz, double sinl, double cosl,
                                             double coslo, double sinlo, double u, double v, double gs,
                                             double alt, double vs, double rpz, double hpz, double tlap) {
  const double ag = fabs(gs) + 0.5e-3;
  const double ht = 0.5 * tlap;
  const double cmax = (rpz + (ag + kVcap + 0.5e-3) * tlap) * (1.0 + 1e-5) * (1.0 / 6.35e6);
  const double rhop = cosl - cmax;
  double mx = px, my = py, mz = pz;
  float s = INFINITY;
  if (fabs(gs) <= kVcap && isfinite(u) && isfinite(v) && rhop >= 0.05 && cmax <= 0.1) {
    const double kb = 1.5707963267948966 + 2.5707963267948966 / rhop;
    const double sm = ((0.5 * rpz + ag * ht) * (1.0 + 1e-5) + 0.012 * (0.5 * rpz + ag * tlap) +
                       ag * ht * kb * cmax) * (1.0 / 6.3e6) + 0.25 * cmax * cmax + 1e-6;
    const double f = ht * (1.0 / 6371000.0);
    mx = px + f * (-u * sinlo - v * sinl * coslo);
    my = py + f * (u * coslo - v * sinl * sinlo);
    mz = pz + f * (v * cosl);
    s = (sm < 0.5) ? (float)sm : INFINITY;
  }
  const double am = alt + vs * ht;
  const double h = (0.5 * hpz + (fabs(vs) + 1.5e-6) * ht) * (1.0 + 1e-5) + 0.5 + 1e-6 * fabs(am);
  PFRec p = make_pf(mx, my, mz, s, am, h);
  p.alt = (float)alt;
  return p;
}

struct SoA6 {
  const double *lat, *lon, *trk, *gs, *alt, *vs;
};

// fp64 column record of aircraft o: intruder[o] geometry, own[o] velocity /
// altitude (the per-aircraft factors of StateBasedCD.py's broadcasts)
// col_record_t: from sin / cos(radians(la)) and u / v a caller already holds
// (bitwise the values col_record_v computes)
__device__ __forceinline__ ColRec col_record_t(double la, double lo, double sinlat, double coslat, double u,
                                               double v, double alt, double vs, double olat) {
  ColRec c;
  c.lat = la;
  c.lon = lo;
  c.sinlat = sinlat;
  c.coslat = coslat;
  c.hemA = fabs(la) * (rwgs84_sc(sinlat, coslat) + kWGS84_A);  // geo.py:127 (rwgs84 of the same radians)
  c.u = u;
  c.v = v;
  c.alt = alt;
  c.vs = vs;
  c.eps = (olat == 0.0) ? 0.000001 : 0.0;      // geo.py:128 (column-indexed)
  c.olat = olat;
  for (int q = 0; q < 5; ++q) c.pad[q] = 0.0;
  return c;
}
__device__ __forceinline__ ColRec col_record_v(double la, double lo, double trkd, double gs, double alt, double vs,
                                               double olat) {
  double sl, cl, st, ct;
  sincos(la * kD2R, &sl, &cl);
  sincos(trkd * kD2R, &st, &ct);
  return col_record_t(la, lo, sl, cl, gs * st, gs * ct, alt, vs, olat);  // u, v: StateBasedCD.py:31-32
}

// the column's inputs to every tcpa of its column (position, velocity) are
// finite: else every tcpa[i, j] is NaN (StateBasedCD.py:58-72) and so is every
// row's tcpamax (:90) -- Ctx::nonfin
__device__ __forceinline__ bool col_tcpa_finite(const ColRec &c) {
  return isfinite(c.lat) && isfinite(c.lon) && isfinite(c.u) && isfinite(c.v);
}

__device__ __forceinline__ ColRec col_record(const SoA6 &own, const SoA6 &intr, int o) {
  return col_record_v(intr.lat[o], intr.lon[o], own.trk[o], own.gs[o], own.alt[o], own.vs[o], own.lat[o]);
}

// One home-ordered record k of the resident sim (presorted, own == intruder,
// shared rows / columns, no candidate-list reuse): exactly k_prep_cols' work
// for that case.  rec: also the 128-B fp64 record.
struct PrepOut {
  ColRec *C;
  PFRec *PC;
  PFVel *PV;
  float4 *PP;
};
// trig (nullable): {sin, cos(radians(la)), gs sin, gs cos(radians(trk))} the
// caller computed with the same expressions (K4': its step's)
__device__ __forceinline__ PFRec prep_home_record(int k, double la, double lo, double trk, double gs, double alt,
                                                  double vs, double rpz, double hpz, double tla, int mid, int rec,
                                                  const PrepOut &out, unsigned long long *nfw,
                                                  unsigned long long nfe, const double *trig = nullptr) {
  const double tlap = tla > 0.0 ? tla : 0.0;
  const ColRec c = trig ? col_record_t(la, lo, trig[0], trig[1], trig[2], trig[3], alt, vs, la)
                        : col_record_v(la, lo, trk, gs, alt, vs, la);
  if (nfw && !col_tcpa_finite(c)) *nfw = nfe;
  if (rec) out.C[k] = c;
  const double sinl = c.sinlat, cosl = c.coslat;
  const double lor = c.lon * kD2R;
  double coslo, sinlo;
  sincos(lor, &sinlo, &coslo);
  const double px = cosl * coslo, py = cosl * sinlo, pz = sinl;
  const float sadd = 0.f, sv = 0.f;
  const PFRec p = mid ? make_pf_mid(px, py, pz, sinl, cosl, coslo, sinlo, c.u, c.v, gs, c.alt, c.vs, rpz, hpz, tlap)
                      : make_pf(px, py, pz, reach_h(rpz, gs, tlap) + sadd, c.alt,
                                reach_v(hpz, c.vs, c.alt, tlap) + (double)sv, sv);
  out.PP[k] = make_float4((float)px, (float)py, (float)pz, 0.f);
  PFVel v;
  v.u = (float)c.u;
  v.v = (float)c.v;
  v.vs = (float)c.vs;
  v.flags = (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) || !(cosl > 1e-2)) ? 1u : 0u;
  out.PC[k] = p;
  out.PV[k] = v;
  return p;
}

__device__ __forceinline__ float xmin(float v, int o) { return fminf(v, __shfl_xor(v, o)); }
__device__ __forceinline__ float xmax(float v, int o) { return fmaxf(v, __shfl_xor(v, o)); }

// Boxes of one kGroup-record group g (one wave, lane = record): its kSub-record
// sub-group boxes to sbox (nullable) and the group box to gbox[g]; returns
// the group box (lane 0).  The lane's record p is passed in registers by the
// lane that just computed it (reading it back from memory put a store ->
// load round trip into K0b and K4'); lanes past cnt pass anything.
__device__ __forceinline__ TileBox group_boxes_v(int cnt, int g, const PFRec &p, TileBox *__restrict__ sbox,
                                                 TileBox *__restrict__ gbox) {
  const int lane = threadIdx.x & 63;
  const int k = g * kGroup + lane;
  const int ngroups = (cnt + kGroup - 1) / kGroup;
  float lo[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, hi[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  float smax = 0.f;
  if (k < cnt) {
    lo[0] = hi[0] = p.x;
    lo[1] = hi[1] = p.y;
    lo[2] = hi[2] = p.z;
    lo[3] = p.lo;
    hi[3] = p.hi;
    smax = p.s == p.s ? p.s : INFINITY;
  }
  auto mkbox = [&](int count) {
    TileBox b;
    for (int q = 0; q < 3; ++q) {
      b.lo[q] = lo[q];
      b.hi[q] = hi[q];
    }
    b.vlo = lo[3];
    b.vhi = hi[3];
    b.smax = smax;
    b.pad0 = 0.f;
    b.count = count;
    b.pad1 = 0;
    return b;
  };
  for (int o = 1; o < kSub; o <<= 1) {  // within each kSub-lane sub-group
    for (int q = 0; q < 4; ++q) {
      lo[q] = xmin(lo[q], o);
      hi[q] = xmax(hi[q], o);
    }
    smax = xmax(smax, o);
  }
  const int sg = g * (kGroup / kSub) + lane / kSub;
  if (sbox && (lane & (kSub - 1)) == 0 && sg * kSub < cnt) sbox[sg] = mkbox(min(kSub, cnt - sg * kSub));
  for (int o = kSub; o < 64; o <<= 1) {
    for (int q = 0; q < 4; ++q) {
      lo[q] = xmin(lo[q], o);
      hi[q] = xmax(hi[q], o);
    }
    smax = xmax(smax, o);
  }
  const TileBox b = mkbox(g < ngroups ? min(kGroup, cnt - g * kGroup) : 0);
  if (lane == 0 && g < ngroups) gbox[g] = b;
  return b;
}
__device__ __forceinline__ TileBox group_boxes(int cnt, int g, const PFRec *__restrict__ P,
                                               TileBox *__restrict__ sbox, TileBox *__restrict__ gbox) {
  const int k = g * kGroup + (threadIdx.x & 63);
  PFRec p{};
  if (k < cnt) p = P[k];
  return group_boxes_v(cnt, g, p, sbox, gbox);
}

// the empty box (the identity of box_union)
__device__ __forceinline__ TileBox empty_box() {
  TileBox b;
  for (int q = 0; q < 3; ++q) {
    b.lo[q] = INFINITY;
    b.hi[q] = -INFINITY;
  }
  b.vlo = INFINITY;
  b.vhi = -INFINITY;
  b.smax = 0.f;
  b.pad0 = 0.f;
  b.count = 0;
  b.pad1 = 0;
  return b;
}

// Boxes of one kTile-record tile (workgroup = kTile lanes, one wave per
// group): group_boxes, then their union to tbox[tile] (in group order).
// Shared by k_boxes and the fused K0b+K0c path of k_prep_cols.
__device__ __forceinline__ void tile_boxes_v(int cnt, int tile, const PFRec &p, TileBox *gb,
                                             TileBox *__restrict__ sbox, TileBox *__restrict__ gbox,
                                             TileBox *__restrict__ tbox) {
  const int w = threadIdx.x >> 6;
  const TileBox b = group_boxes_v(cnt, tile * kGroupsPerTile + w, p, sbox, gbox);
  if ((threadIdx.x & 63) == 0) gb[w] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    TileBox u = gb[0];
    for (int q = 1; q < kGroupsPerTile; ++q) u = box_union(u, gb[q]);
    tbox[tile] = u;
  }
}
__device__ __forceinline__ void tile_boxes(int cnt, int tile, const PFRec *__restrict__ P, TileBox *gb,
                                           TileBox *__restrict__ sbox, TileBox *__restrict__ gbox,
                                           TileBox *__restrict__ tbox) {
  const int k = tile * kTile + (int)threadIdx.x;
  PFRec p{};
  if (k < cnt) p = P[k];
  tile_boxes_v(cnt, tile, p, gb, sbox, gbox, tbox);
}

// tbox[t] from the group boxes of tile t (K0z after a K4' that wrote the group
// boxes): the same union, in the same order, as tile_boxes (missing trailing
// groups are empty boxes there too)
__device__ __forceinline__ void tile_from_groups(int cnt, int t, const TileBox *__restrict__ gbox,
                                                 TileBox *__restrict__ tbox) {
  const int ngroups = (cnt + kGroup - 1) / kGroup;
  const int g0 = t * kGroupsPerTile;
  TileBox u = g0 < ngroups ? gbox[g0] : empty_box();
  for (int q = 1; q < kGroupsPerTile; ++q) u = box_union(u, g0 + q < ngroups ? gbox[g0 + q] : empty_box());
  tbox[t] = u;
}

}  // namespace bsa
