// StateBased conflict detection for gfx950:
//   StateBasedCD.detect (bluesky/traffic/asas/StateBasedCD.py:7-103) with
//   geo.qdrdist_matrix (bluesky/tools/geo.py:110-162) fused in.
//
// Pipeline, all on one stream, one host sync:
//   K0a keys       Morton code of each position's unit vector (rows = own,
//                  columns = intruder), then hipcub radix sort -> spatial order.
//   K0b prep       per sorted index: fp64 records (the per-aircraft factors of
//                  the reference's N x N broadcasts) + fp32 prefilter records.
//   K0c tilebox    bounds of every 512-row block / 512-column tile.
//   K0d tilepairs  (row block, column tile) pairs whose bounds can contain a
//                  kept pair; all others are skipped without touching a pair.
//   K1a prefilter  N-body sweep of the surviving tile pairs: lane = ownship
//                  row (2 per lane), column tile in LDS (broadcast reads);
//                  stage 1 conservative reach test, stage 2 conservative
//                  fp32 closest-approach refine (exact-safe proofs);
//                  survivors compacted per wave (ballot/mbcnt, 1 atomic/flush).
//   K1b exact      one lane per candidate: the reference's fp64 expression
//                  sequence op for op (-ffp-contract=off), outputs appended
//                  with one atomic per wave.
//   K2  sort       radix sort on (i << 32 | j) = the reference's row-major
//                  np.where order, then a gather.
// Neither the spatial order nor the culling changes any result: every stage
// before K1b only removes pairs that provably cannot be a conflict or a loss
// of separation, and K1b evaluates the survivors exactly.
#include <hipcub/hipcub.hpp>

#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

// ------------------------------------------------------------------ math
// numpy.maximum / numpy.minimum semantics: NaN propagates, ties keep `a`.
__device__ __forceinline__ double np_max(double a, double b) {
  return (a >= b || a != a) ? a : b;
}
__device__ __forceinline__ double np_min(double a, double b) {
  return (a <= b || a != a) ? a : b;
}

// geo.py:32-54 rwgs84_matrix, elementwise, same op order.
__device__ __forceinline__ double rwgs84(double latd) {
  const double a = kWGS84_A, b = kWGS84_B;
  const double lat = latd * kD2R;
  const double coslat = cos(lat);
  const double sinlat = sin(lat);
  const double an = (a * a) * coslat;
  const double bn = (b * b) * sinlat;
  const double ad = a * coslat;
  const double bd = b * sinlat;
  const double anan = an * an;
  const double bnbn = bn * bn;
  const double adad = ad * ad;
  const double bdbd = bd * bd;
  return sqrt((anan + bnbn) / (adad + bdbd));
}

// ------------------------------------------------------------------ K0a keys
__device__ __forceinline__ unsigned expand10(unsigned v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}
__device__ __forceinline__ unsigned morton_latlon(double latd, double lond) {
  const double la = latd * kD2R, lo = lond * kD2R;
  const double cl = cos(la);
  const double p[3] = {cl * cos(lo), cl * sin(lo), sin(la)};
  unsigned key = 0;
  for (int k = 0; k < 3; ++k) {
    if (!(p[k] == p[k]) || isinf(p[k])) return 0xffffffffu;
    int q = (int)((p[k] + 1.0) * 512.0);
    q = q < 0 ? 0 : (q > 1023 ? 1023 : q);
    key |= expand10((unsigned)q) << (2 - k);
  }
  return key;
}

__global__ __launch_bounds__(256) void k_keys(int cnt, int base, const double *__restrict__ lat,
                                              const double *__restrict__ lon,
                                              unsigned *__restrict__ key,
                                              unsigned *__restrict__ idx) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const int o = base + k;
  key[k] = morton_latlon(lat[o], lon[o]);
  idx[k] = (unsigned)o;
}

// ------------------------------------------------------------------ K0b prep
__device__ __forceinline__ float reach_h(double rpz, double gs, double tlap) {
  // horizontal half-bound in unit-sphere chord units: a pair is kept iff
  // chord < s_i + s_j,  s = ((R/2 + (|gs| + 0.5e-3) tla)(1 + 1e-5)) / 6.3e6 + 1e-6
  const double s = ((0.5 * rpz + (fabs(gs) + 0.5e-3) * tlap) * (1.0 + 1e-5)) / 6.3e6 + 1e-6;
  return isfinite(s) ? (float)s : INFINITY;
}
__device__ __forceinline__ float reach_v(double hpz, double vs, double alt, double tlap) {
  const double h = (0.5 * hpz + (fabs(vs) + 0.5e-6) * tlap) * (1.0 + 1e-5) + 0.5 + 1e-6 * fabs(alt);
  return isfinite(h) ? (float)h : INFINITY;
}

struct SoA6 {
  const double *lat, *lon, *trk, *gs, *alt, *vs;
};

// Row records, sorted position k -> original row perm[k]: own[i] geometry,
// intruder[i] velocity / altitude (StateBasedCD.py:39-40,65-69 orientation).
__global__ __launch_bounds__(256) void k_prep_rows(int cnt, const unsigned *__restrict__ perm,
                                                   SoA6 own, SoA6 intr, double rpz, double hpz,
                                                   double tla, RowRec *__restrict__ R,
                                                   PFRec *__restrict__ PR, PFAux *__restrict__ PA) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const int o = (int)perm[k];
  const double tlap = tla > 0.0 ? tla : 0.0;
  const double la = own.lat[o], lo = own.lon[o];
  const double rad = la * kD2R;
  const double sinl = sin(rad), cosl = cos(rad);
  const double trk = intr.trk[o] * kD2R;
  const double gs = intr.gs[o];
  RowRec r;
  r.lat = la;
  r.lon = lo;
  r.sinlat = sinl;
  r.coslat = cosl;
  r.hemA = fabs(la) * (rwgs84(la) + kWGS84_A);  // geo.py:127
  r.u = gs * sin(trk);                           // StateBasedCD.py:36-37
  r.v = gs * cos(trk);
  r.alt = intr.alt[o];
  r.vs = intr.vs[o];
  for (int q = 0; q < 7; ++q) r.pad[q] = 0.0;
  R[k] = r;
  const double lor = lo * kD2R;
  PFRec p;
  p.x = (float)(cosl * cos(lor));
  p.y = (float)(cosl * sin(lor));
  p.z = (float)sinl;
  p.s = reach_h(rpz, gs, tlap);
  p.alt = (float)r.alt;
  p.h = reach_v(hpz, r.vs, r.alt, tlap);
  p.u = (float)r.u;
  p.v = (float)r.v;
  PFAux a;
  a.vs = (float)r.vs;
  a.flags = 0;
  // local east / north basis of the CPA refine (fp64, then rounded)
  // e = (-sin lon, cos lon, 0), n = (-sin lat cos lon, -sin lat sin lon, cos lat)
  const double slo = sin(lor), clo = cos(lor);
  a.ex = (float)(-slo);
  a.ey = (float)clo;
  a.nx = (float)(-sinl * clo);
  a.ny = (float)(-sinl * slo);
  a.nz = (float)cosl;
  a.pad = 0.f;
  if (!(cosl > 1e-2)) a.flags = 1;  // within ~0.6 deg of a pole (or |lat| > 90): never refine
  if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) {
    p.s = INFINITY;
    a.flags = 1;
  }
  PR[k] = p;
  PA[k] = a;
}

// Column records: intruder[j] geometry, own[j] velocity / altitude.
__global__ __launch_bounds__(256) void k_prep_cols(int cnt, const unsigned *__restrict__ perm,
                                                   SoA6 own, SoA6 intr, int distinct, double rpz,
                                                   double hpz, double tla, ColRec *__restrict__ C,
                                                   PFRec *__restrict__ PC, PFAux *__restrict__ PA) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const int o = (int)perm[k];
  const double tlap = tla > 0.0 ? tla : 0.0;
  const double la = intr.lat[o], lo = intr.lon[o];
  const double rad = la * kD2R;
  const double sinl = sin(rad), cosl = cos(rad);
  const double trk = own.trk[o] * kD2R;
  const double gs = own.gs[o];
  const double olat = own.lat[o];
  ColRec c;
  c.lat = la;
  c.lon = lo;
  c.sinlat = sinl;
  c.coslat = cosl;
  c.hemA = fabs(la) * (rwgs84(la) + kWGS84_A);
  c.u = gs * sin(trk);                           // StateBasedCD.py:31-32
  c.v = gs * cos(trk);
  c.alt = own.alt[o];
  c.vs = own.vs[o];
  c.eps = (olat == 0.0) ? 0.000001 : 0.0;       // geo.py:128 (column-indexed)
  for (int q = 0; q < 6; ++q) c.pad[q] = 0.0;
  C[k] = c;
  const double lor = lo * kD2R;
  PFRec p;
  p.x = (float)(cosl * cos(lor));
  p.y = (float)(cosl * sin(lor));
  p.z = (float)sinl;
  p.s = reach_h(rpz, gs, tlap);
  p.alt = (float)c.alt;
  p.h = reach_v(hpz, c.vs, c.alt, tlap);
  p.u = (float)c.u;
  p.v = (float)c.v;
  PFAux a;
  a.vs = (float)c.vs;
  a.flags = 0;
  a.ex = a.ey = a.nx = a.ny = a.nz = a.pad = 0.f;  // the refine uses the row's basis only
  // (own.lat[j] == 0) leaves the different-hemisphere radius unbounded below
  // when own != intruder (geo.py:128): never prune or refine such a column.
  if ((distinct && olat == 0.0) || !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) {
    p.s = INFINITY;
    a.flags = 1;
  }
  PC[k] = p;
  PA[k] = a;
}

// ------------------------------------------------------------------ K0c tile boxes
__device__ __forceinline__ float wmin(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wmax(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Bounds of every group of kGroup (= one wave's 64 lanes) consecutive sorted
// records: one wave per group, lane = record.  NaN coordinates drop out of
// the min/max (fminf/fmaxf), which is safe: a record with a NaN coordinate
// never passes the reach test.
constexpr int kGroup = 64;
static_assert(kTile % kGroup == 0, "tiles are whole groups");

__global__ __launch_bounds__(256) void k_groupbox(int cnt, const PFRec *__restrict__ P,
                                                  TileBox *__restrict__ box) {
  const int g = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  const int k = g * kGroup + lane;
  const int ngroups = (cnt + kGroup - 1) / kGroup;
  if (g >= ngroups) return;  // whole wave exits together
  float lo[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, hi[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  float smax = 0.f, hmax = 0.f;
  if (k < cnt) {
    const PFRec p = P[k];
    lo[0] = hi[0] = p.x;
    lo[1] = hi[1] = p.y;
    lo[2] = hi[2] = p.z;
    lo[3] = hi[3] = p.alt;
    smax = p.s == p.s ? p.s : INFINITY;
    hmax = p.h == p.h ? p.h : INFINITY;
  }
  for (int q = 0; q < 4; ++q) {
    lo[q] = wmin(lo[q]);
    hi[q] = wmax(hi[q]);
  }
  smax = wmax(smax);
  hmax = wmax(hmax);
  if (lane == 0) {
    TileBox b;
    for (int q = 0; q < 3; ++q) {
      b.lo[q] = lo[q];
      b.hi[q] = hi[q];
    }
    b.altlo = lo[3];
    b.althi = hi[3];
    b.smax = smax;
    b.hmax = hmax;
    b.count = min(kGroup, cnt - g * kGroup);
    b.pad = 0;
    box[g] = b;
  }
}

__device__ __forceinline__ TileBox box_union(const TileBox &a, const TileBox &b) {
  TileBox u;
  for (int q = 0; q < 3; ++q) {
    u.lo[q] = fminf(a.lo[q], b.lo[q]);
    u.hi[q] = fmaxf(a.hi[q], b.hi[q]);
  }
  u.altlo = fminf(a.altlo, b.altlo);
  u.althi = fmaxf(a.althi, b.althi);
  u.smax = fmaxf(a.smax, b.smax);
  u.hmax = fmaxf(a.hmax, b.hmax);
  u.count = a.count + b.count;
  u.pad = 0;
  return u;
}

// tile box = union of its kTile / kGroup group boxes
__global__ __launch_bounds__(256) void k_tileunion(int ntiles, int ngroups, const TileBox *__restrict__ g,
                                                   TileBox *__restrict__ t) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ntiles) return;
  const int g0 = k * (kTile / kGroup), g1 = min(ngroups, g0 + kTile / kGroup);
  TileBox u = g[g0];
  for (int q = g0 + 1; q < g1; ++q) u = box_union(u, g[q]);
  t[k] = u;
}

// ------------------------------------------------------------------ K0d tile pairs
__device__ __forceinline__ float gap(float alo, float ahi, float blo, float bhi) {
  return fmaxf(0.f, fmaxf(alo - bhi, blo - ahi));
}

__global__ __launch_bounds__(256) void k_tilepairs(int nrt, int nct, const TileBox *__restrict__ rb,
                                                   const TileBox *__restrict__ cb, int noprune,
                                                   uint2 *__restrict__ out,
                                                   unsigned long long *__restrict__ count) {
  const long long id = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = id < (long long)nrt * nct;
  bool keep = false;
  int rt = 0, ct = 0;
  if (valid) {
    rt = (int)(id / nct);
    ct = (int)(id % nct);
    if (noprune) {
      keep = true;
    } else {
      const TileBox a = rb[rt], b = cb[ct];
      const float gx = gap(a.lo[0], a.hi[0], b.lo[0], b.hi[0]);
      const float gy = gap(a.lo[1], a.hi[1], b.lo[1], b.hi[1]);
      const float gz = gap(a.lo[2], a.hi[2], b.lo[2], b.hi[2]);
      const float d2 = gx * gx + gy * gy + gz * gz;
      const float st = (a.smax + b.smax) * 1.00001f + 1e-6f;
      const float ga = gap(a.altlo, a.althi, b.altlo, b.althi);
      // a pair inside can pass only if its chord < s_i + s_j <= smax_a + smax_b
      // and |dalt| < h_i + h_j <= hmax_a + hmax_b; the gaps bound chord/dalt below
      keep = !(d2 >= st * st) && !(ga >= (a.hmax + b.hmax) * 1.00001f + 1e-3f);
    }
  }
  const unsigned long long m = __ballot(keep);
  if (m) {
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(m));
    base = __shfl(base, leader);
    if (keep) {
      const unsigned pos = (unsigned)(base + __builtin_amdgcn_mbcnt_hi(
                                                 (unsigned)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)));
      out[pos] = make_uint2((unsigned)rt, (unsigned)ct);
    }
  }
}

// ------------------------------------------------------------------ K1a prefilter
constexpr int PF_BLOCK = 256;
constexpr int PF_WAVES = PF_BLOCK / 64;
static_assert(kTile == 2 * PF_BLOCK, "2 rows per lane");

struct RefineParams {
  float R;      // rpz [m]
  float H;      // hpz [m]
  float T;      // max(tla, 0) [s]
  float lim2;   // ((R + EABS) / (1 - E1))^2
};
constexpr float kRS = 6371000.f;   // scale of the unit-sphere chord to metres
constexpr float kE1 = 0.012f;      // bound on |log(reference dist / estimated dist)|
constexpr float kEABS = 50.f;      // absolute position error budget [m]

__device__ __forceinline__ unsigned lane_prefix(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ unsigned long long wave_bcast_u64(unsigned long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

typedef float f2 __attribute__((ext_vector_type(2)));

// stage 2: conservative closest-approach refine of one (row, column) pair.
// Returns false only when no t in [0, max(tla,0)] can lie in both the
// vertical and the horizontal window of the reference's geometry
// (DESIGN.md "CPA refine"); any NaN keeps the pair.
__device__ __forceinline__ bool pf_refine(const PFRec &r, const PFAux &ra, const PFRec &c,
                                          const PFAux &ca, const RefineParams &rp) {
  // flags: row basis unusable (pole), quirk columns, non-finite positions
  if (ra.flags | ca.flags) return true;
  const float dx = c.x - r.x, dy = c.y - r.y, dz = c.z - r.z;
  if (dx * dx + dy * dy + dz * dz > 0.04f) return true;   // > ~1270 km: keep, no refine
  // chord projected on the row's local east / north basis (precomputed in prep)
  const float pe = (dx * ra.ex + dy * ra.ey) * kRS;
  const float pn = (dx * ra.nx + dy * ra.ny + dz * ra.nz) * kRS;
  const float ve = c.u - r.u, vn = c.v - r.v;              // own.u[j] - int.u[i]
  const float vv = ve * ve + vn * vn;
  if (!(vv >= 4e-6f)) return true;                         // reference may clamp dv2
  const float dalt = c.alt - r.alt;                        // own.alt[j] - int.alt[i]
  const float dvs = ca.vs - ra.vs;
  const float adv = __builtin_fabsf(dvs);
  float t0 = 0.f, t1 = rp.T;
  // reciprocals by v_rcp_f32 (1 ulp): every division here only places a
  // window edge or the closest-approach time, and the margins below are
  // many orders of magnitude wider than 1 ulp
  if (adv < 1e-3f) {
    if (__builtin_fabsf(dalt) >= rp.H + 1e-3f * rp.T + 2.f + 1e-5f * __builtin_fabsf(dalt)) return false;
  } else {
    const float inv = __builtin_amdgcn_rcpf(dvs);
    const float ta = (-rp.H - dalt) * inv, tb = (rp.H - dalt) * inv;
    const float lo = fminf(ta, tb), hi = fmaxf(ta, tb);
    const float d = (2.f + 1e-5f * (__builtin_fabsf(dalt) + rp.H)) * __builtin_fabsf(inv) +
                    1e-4f * fmaxf(__builtin_fabsf(lo), __builtin_fabsf(hi));
    t0 = fmaxf(lo - d, 0.f);
    t1 = fminf(hi + d, rp.T);
    if (t0 > t1) return false;
  }
  const float tl = t0 * (1.f - kE1), th = t1 * (1.f + 2.f * kE1);
  float ts = -(pe * ve + pn * vn) * __builtin_amdgcn_rcpf(vv);
  ts = fminf(fmaxf(ts, tl), th);
  const float qe = pe + ve * ts, qn = pn + vn * ts;
  return !(qe * qe + qn * qn > rp.lim2);
}

// can any pair of the two boxes pass the reach test?  (gap bounds the chord /
// |dalt| from below; s_i + s_j <= smax_a + smax_b, h_i + h_j <= hmax_a + hmax_b)
__device__ __forceinline__ bool boxes_may_interact(const TileBox &a, const TileBox &b) {
  const float gx = gap(a.lo[0], a.hi[0], b.lo[0], b.hi[0]);
  const float gy = gap(a.lo[1], a.hi[1], b.lo[1], b.hi[1]);
  const float gz = gap(a.lo[2], a.hi[2], b.lo[2], b.hi[2]);
  const float d2 = gx * gx + gy * gy + gz * gz;
  const float st = (a.smax + b.smax) * 1.00001f + 1e-6f;
  const float ga = gap(a.altlo, a.althi, b.altlo, b.althi);
  return !(d2 >= st * st) && !(ga >= (a.hmax + b.hmax) * 1.00001f + 1e-3f);
}

constexpr int PF_Q1 = 1024;  // per-wave stage-1 queue: u32 (row_local << 16 | col_local)
constexpr int PF_Q2 = 256;   // per-wave stage-2 queue: uint2 (sorted row, sorted column)
constexpr int PF_WROWS = 128;  // rows per wave (2 per lane)
constexpr int kWorkShards = 8;   // one dequeue counter per XCD group
constexpr int kWorkStride = 16;  // u64 words between counters (128 B apart)
static_assert(PF_WAVES * PF_WROWS == kTile, "4 waves x 128 rows = one row block");

__device__ __forceinline__ void pf_flush(uint2 *q, unsigned qn, int lane, uint2 *__restrict__ cand,
                                         unsigned long long *__restrict__ count,
                                         unsigned long long cap) {
  __builtin_amdgcn_wave_barrier();
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(count, (unsigned long long)qn);
  base = wave_bcast_u64(base);
  for (unsigned k = lane; k < qn; k += 64)
    if (base + k < cap) cand[base + k] = q[k];
  __builtin_amdgcn_wave_barrier();
}

// K1a: each wave sweeps its 128 rows against the 512 columns of a tile pair
// in 64-column groups (a group is skipped when the wave's row box and the
// group box cannot interact).  Stage 1 (packed fp32 reach test, 2 rows per
// lane) pushes survivors into an LDS queue; the queue is drained with all 64
// lanes busy through stage 2 (refine), whose survivors go to a second queue
// that is flushed to HBM with one atomic per flush.
template <bool NOPRUNE>
__global__ __launch_bounds__(PF_BLOCK) void k_prefilter(
    const PFRec *__restrict__ prow, const PFAux *__restrict__ arow, int nrows,
    const PFRec *__restrict__ pcol, const PFAux *__restrict__ acol, int ncols,
    const TileBox *__restrict__ gbox_r, const TileBox *__restrict__ gbox_c,
    const uint2 *__restrict__ tiles, Counters *__restrict__ cnt,
    unsigned long long *__restrict__ work, RefineParams rp,
    uint2 *__restrict__ cand, unsigned long long cap) {
  __shared__ unsigned q1s[PF_WAVES][PF_Q1];
  __shared__ uint2 q2s[PF_WAVES][PF_Q2];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned long long ntiles = cnt->tiles;
  unsigned *q1 = q1s[w];
  uint2 *q2 = q2s[w];
  unsigned n2 = 0;        // wave-uniform
  unsigned groups = 0;    // 64-column groups swept by this wave (for the roofline)
  const float qnan = __builtin_nanf("");
  // Dynamic work distribution: an item is one (tile pair, 128-row slice);
  // each wave dequeues items from the counter of its XCD group (blockIdx % 8)
  // so no single word takes every dequeue (MI355X_MICROARCH 'dequeue').
  const unsigned long long nitems = ntiles * PF_WAVES;
  const unsigned shard = blockIdx.x & (kWorkShards - 1);
  unsigned long long *wq = work + shard * kWorkStride;
  for (;;) {
    unsigned long long m = 0;
    if (lane == 0) m = atomicAdd(wq, 1ull);
    const unsigned long long item = wave_bcast_u64(m) * kWorkShards + shard;
    if (item >= nitems) break;
    const uint2 rc = tiles[item / PF_WAVES];
    const int rbase = (int)rc.x * kTile + (int)(item % PF_WAVES) * PF_WROWS;
    if (rbase >= nrows) continue;
    const int cbase = (int)rc.y * kTile;
    const int ka_row = rbase + lane, kb_row = rbase + 64 + lane;
    const bool va = ka_row < nrows, vb = kb_row < nrows;
    PFRec A, B;
    if (va) A = prow[ka_row]; else { A.x = A.y = A.z = qnan; A.s = A.alt = A.h = A.u = A.v = 0.f; }
    if (vb) B = prow[kb_row]; else { B.x = B.y = B.z = qnan; B.s = B.alt = B.h = B.u = B.v = 0.f; }
    const f2 X = {A.x, B.x}, Y = {A.y, B.y}, Z = {A.z, B.z};
    const f2 S = {A.s, B.s}, AL = {A.alt, B.alt}, HH = {A.h, B.h};
    TileBox rbx = gbox_r[rbase / kGroup];
    if (rbase + 64 < nrows) rbx = box_union(rbx, gbox_r[rbase / kGroup + 1]);
    unsigned n1 = 0;  // wave-uniform
    const int ng = min(kTile / kGroup, (ncols - cbase + kGroup - 1) / kGroup);

    auto drain = [&]() {
      __builtin_amdgcn_wave_barrier();
      for (unsigned b0 = 0; b0 < n1; b0 += 64) {
        const unsigned k = b0 + lane;
        bool keep = false;
        unsigned gi = 0, gj = 0;
        if (k < n1) {
          const unsigned e = q1[k];
          gi = (unsigned)rbase + (e >> 16);
          gj = (unsigned)cbase + (e & 0xffffu);
          keep = NOPRUNE ? true : pf_refine(prow[gi], arow[gi], pcol[gj], acol[gj], rp);
        }
        const unsigned long long m = __ballot(keep);
        if (m) {
          if (keep) q2[n2 + lane_prefix(m)] = make_uint2(gi, gj);
          n2 = __builtin_amdgcn_readfirstlane(n2 + (unsigned)__popcll(m));
          if (n2 > (unsigned)(PF_Q2 - 64)) {
            pf_flush(q2, n2, lane, cand, &cnt->cand, cap);
            n2 = 0;
          }
        }
      }
      n1 = 0;
      __builtin_amdgcn_wave_barrier();
    };

    // stage 1 for one column record, packed over the lane's two rows; the
    // survivors of an 8-column chunk accumulate as per-lane bit masks and are
    // queued once per chunk (one wave prefix sum instead of per-column ballots)
    auto reach = [&](const PFRec &c, bool &ka, bool &kb) {
      if (NOPRUNE) {
        ka = va;
        kb = vb;
      } else {
        const f2 dx = (f2){c.x, c.x} - X, dy = (f2){c.y, c.y} - Y, dz = (f2){c.z, c.z} - Z;
        f2 d2 = dx * dx;
        d2 = __builtin_elementwise_fma(dy, dy, d2);
        d2 = __builtin_elementwise_fma(dz, dz, d2);
        const f2 st = S + (f2){c.s, c.s};
        const f2 st2 = st * st;
        const f2 dh = (f2){c.alt, c.alt} - AL;
        const f2 hh = HH + (f2){c.h, c.h};
        ka = (d2.x < st2.x) & (__builtin_fabsf(dh.x) < hh.x);
        kb = (d2.y < st2.y) & (__builtin_fabsf(dh.y) < hh.y);
      }
    };
    auto enqueue = [&](unsigned ba, unsigned bb, unsigned col0) {
      const unsigned cnt = (unsigned)__popc(ba) + (unsigned)__popc(bb);
      if (!__ballot(cnt != 0)) return;
      unsigned x = cnt;  // inclusive wave prefix sum of cnt
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      const unsigned total = __builtin_amdgcn_readlane(x, 63);
      if (n1 + total > (unsigned)PF_Q1) drain();  // total <= 2 * 64 * 8 = PF_Q1
      unsigned pos = n1 + x - cnt;
      while (ba) {
        q1[pos++] = ((unsigned)lane << 16) | (col0 + (unsigned)__builtin_ctz(ba));
        ba &= ba - 1;
      }
      while (bb) {
        q1[pos++] = ((unsigned)(64 + lane) << 16) | (col0 + (unsigned)__builtin_ctz(bb));
        bb &= bb - 1;
      }
      n1 = __builtin_amdgcn_readfirstlane(n1 + total);
    };

    for (int g = 0; g < ng; ++g) {
      const int c0 = cbase + g * kGroup;
      if (!NOPRUNE && !boxes_may_interact(rbx, gbox_c[c0 / kGroup])) continue;
      ++groups;
      const int nc = min(kGroup, ncols - c0);
      const unsigned cl0 = (unsigned)(g * kGroup);
      if (nc == kGroup) {
        for (int j0 = 0; j0 < kGroup; j0 += 8) {
          unsigned ba = 0, bb = 0;
#pragma unroll
          for (int h4 = 0; h4 < 8; h4 += 4) {
            PFRec cc[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) cc[u] = pcol[c0 + j0 + h4 + u];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              bool ka, kb;
              reach(cc[u], ka, kb);
              ba |= (unsigned)ka << (h4 + u);
              bb |= (unsigned)kb << (h4 + u);
            }
          }
          enqueue(ba, bb, cl0 + (unsigned)j0);
        }
      } else {
        for (int j0 = 0; j0 < nc; j0 += 8) {
          unsigned ba = 0, bb = 0;
          for (int u = 0; u < 8 && j0 + u < nc; ++u) {
            bool ka, kb;
            reach(pcol[c0 + j0 + u], ka, kb);
            ba |= (unsigned)ka << u;
            bb |= (unsigned)kb << u;
          }
          enqueue(ba, bb, cl0 + (unsigned)j0);
        }
      }
    }
    if (n1) drain();
  }
  if (n2) pf_flush(q2, n2, lane, cand, &cnt->cand, cap);
  if (lane == 0 && groups) atomicAdd(&cnt->groups, (unsigned long long)groups);
}

// ------------------------------------------------------------------ K1b exact
struct PairResult {
  bool conf, los;
  double qdr, dist, tcpa, tin, dcpa;
};

// One (i, j) entry of StateBasedCD.detect + geo.qdrdist_matrix, i != j.
__device__ __forceinline__ PairResult eval_pair(const RowRec &r, const ColRec &c, double rpz,
                                                double hpz, double tla) {
  PairResult o;
  // ---- geo.qdrdist_matrix (geo.py:118-160)
  const double prodla = r.lat * c.lat;
  double rr;
  if (prodla < 0) {
    // different hemisphere (geo.py:126-129)
    rr = (0.5 * (r.hemA + c.hemA)) / (fabs(r.lat) + (fabs(c.lat) + c.eps));
  } else {
    rr = rwgs84(r.lat + c.lat);  // geo.py:122: radius at the SUM of the latitudes
  }
  const double diff_lat = c.lat - r.lat;
  const double diff_lon = c.lon - r.lon;
  const double sin1 = diff_lat * kD2R;
  const double sin2 = diff_lon * kD2R;
  const double sin21 = sin(sin2);
  const double cos21 = cos(sin2);
  const double y = sin21 * c.coslat;
  const double x1 = r.coslat * c.sinlat;
  const double x2 = r.sinlat * c.coslat;
  const double x3 = x2 * cos21;
  const double x = x1 - x3;
  const double qdr = atan2(y, x) * kR2D;
  const double sin10 = fabs(sin(sin1 / 2.));
  const double sin20 = fabs(sin(sin2 / 2.));
  const double sin1sin1 = sin10 * sin10;
  const double sin2sin2 = sin20 * sin20;
  const double hav = sin1sin1 + (r.coslat * c.coslat) * sin2sin2;
  const double dist_c = 2. * atan2(sqrt(hav), sqrt(1 - hav));
  const double dist_nm = (rr / kNM) * dist_c;

  // ---- StateBasedCD.detect (StateBasedCD.py:22-83), off-diagonal entry
  const double dist = dist_nm * kNM + 0.0;
  const double qdrrad = qdr * kD2R;
  const double dx = dist * sin(qdrrad);
  const double dy = dist * cos(qdrrad);
  const double du = c.u - r.u;  // own.u[j] - int.u[i]
  const double dv = c.v - r.v;
  double dv2 = du * du + dv * dv;
  dv2 = (fabs(dv2) < 1e-6) ? 1e-6 : dv2;
  const double vrel = sqrt(dv2);
  const double tcpa = -(du * dx + dv * dy) / dv2 + 0.0;
  const double dcpa2 = dist * dist - tcpa * tcpa * dv2;
  const double R2 = rpz * rpz;
  const bool swhorconf = dcpa2 < R2;
  const double dxinhor = sqrt(np_max(0., R2 - dcpa2));
  const double dtinhor = dxinhor / vrel;
  const double tinhor = swhorconf ? tcpa - dtinhor : 1e8;
  const double touthor = swhorconf ? tcpa + dtinhor : -1e8;
  const double dalt = c.alt - r.alt + 0.0;  // own.alt[j] - int.alt[i]
  double dvs = c.vs - r.vs;
  dvs = (fabs(dvs) < 1e-6) ? 1e-6 : dvs;
  const double tcrosshi = (dalt + hpz) / -dvs;
  const double tcrosslo = (dalt - hpz) / -dvs;
  const double tinver = np_min(tcrosshi, tcrosslo);
  const double toutver = np_max(tcrosshi, tcrosslo);
  const double tinconf = np_max(tinver, tinhor);
  const double toutconf = np_min(toutver, touthor);
  o.conf = swhorconf && (tinconf <= toutconf) && (toutconf > 0.0) && (tinconf < tla);
  o.los = (dist < rpz) && (fabs(dalt) < hpz);  // StateBasedCD.py:94
  o.qdr = qdr;
  o.dist = dist;
  o.tcpa = tcpa;
  o.tin = tinconf;
  o.dcpa = sqrt(np_max(dcpa2, 0.0));
  return o;
}

// Results are stored per candidate (flag, key, payload) rather than appended
// to a shared list: appending needs an atomic with return on ONE counter per
// wave, which serialises at ~88/us (MI355X_MICROARCH 'dequeue') and cost
// ~70 us at 100k.  The per-row counts feed K2's counting sort.
__global__ __launch_bounds__(256) void k_exact(
    const RowRec *__restrict__ R, const ColRec *__restrict__ C,
    const unsigned *__restrict__ perm_r, const unsigned *__restrict__ perm_c,
    const uint2 *__restrict__ cand, const unsigned long long *__restrict__ ncand_p,
    unsigned long long cap, double rpz, double hpz, double tla, int rb, int nrows,
    unsigned char *__restrict__ cflag, unsigned long long *__restrict__ ckey,
    double *__restrict__ cpay, unsigned char *__restrict__ inconf,
    unsigned long long *__restrict__ tcpamax_bits, unsigned *__restrict__ rowcnt) {
  const unsigned long long ncand = min(*ncand_p, cap);
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long idx = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
       idx < ncand; idx += stride) {
    const uint2 p = cand[idx];
    const unsigned oi = perm_r[p.x], oj = perm_c[p.y];
    unsigned char flag = 0;
    if (oi != oj) {
      const PairResult o = eval_pair(R[p.x], C[p.y], rpz, hpz, tla);
      flag = (o.conf ? 1 : 0) | (o.los ? 2 : 0);
      const int row = (int)oi - rb;
      if (flag) ckey[idx] = ((unsigned long long)oi << 32) | oj;
      if (o.conf) {
        cpay[0 * cap + idx] = o.qdr;
        cpay[1 * cap + idx] = o.dist;
        cpay[2 * cap + idx] = o.tcpa;
        cpay[3 * cap + idx] = o.tin;
        cpay[4 * cap + idx] = o.dcpa;
        inconf[row] = 1;
        // tcpamax = max_j(tcpa * swconfl) >= +-0 (StateBasedCD.py:90): only
        // positive tcpa can raise it, and positive doubles order as integers.
        if (o.tcpa > 0.0)
          atomicMax(&tcpamax_bits[row], (unsigned long long)__double_as_longlong(o.tcpa));
        atomicAdd(&rowcnt[row], 1u);
      }
      if (o.los) atomicAdd(&rowcnt[nrows + 1 + row], 1u);
    }
    cflag[idx] = flag;
  }
}

// ------------------------------------------------------------------ K2 canonical order
// Per-row counting sort.  rowcnt holds [conflicts per row | 0 | LoS per row | 0]
// (2 * (nrows + 1) words); its exclusive scan gives each row's segment in the
// conflict list and (minus P) in the LoS list.  Pairs are scattered into their
// row segment, then one lane per row sorts its (short) segment by column:
// the result is exactly np.where's row-major order (StateBasedCD.py:93-95).
__global__ __launch_bounds__(256) void k_scatter(const unsigned long long *__restrict__ ncand_p,
                                                 unsigned long long cap, int rb, int nrows,
                                                 const unsigned char *__restrict__ cflag,
                                                 const unsigned long long *__restrict__ ckey,
                                                 const unsigned *__restrict__ rowoff,
                                                 unsigned *__restrict__ rowcnt,
                                                 unsigned *__restrict__ cslot,
                                                 unsigned *__restrict__ lslot) {
  const unsigned long long ncand = min(*ncand_p, cap);
  const unsigned P = rowoff[nrows];
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long k = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; k < ncand;
       k += stride) {
    const unsigned char f = cflag[k];
    if (!f) continue;
    const int row = (int)(ckey[k] >> 32) - rb;
    if (f & 1) {
      const unsigned pos = rowoff[row] + atomicSub(&rowcnt[row], 1u) - 1u;
      cslot[pos] = (unsigned)k;
    }
    if (f & 2) {
      const int r = nrows + 1 + row;
      const unsigned pos = rowoff[r] - P + atomicSub(&rowcnt[r], 1u) - 1u;
      lslot[pos] = (unsigned)k;
    }
  }
}

__global__ __launch_bounds__(256) void k_rowsort(int nrows, int64_t P, const unsigned *__restrict__ rowoff,
                                                 const unsigned long long *__restrict__ ckey,
                                                 unsigned *__restrict__ cslot,
                                                 const double *__restrict__ cpay, unsigned long long cap,
                                                 unsigned *__restrict__ lslot, int *__restrict__ ci,
                                                 int *__restrict__ cj, double *__restrict__ out,
                                                 int *__restrict__ li, int *__restrict__ lj) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  // conflicts of row r
  {
    const unsigned b = rowoff[r], e = rowoff[r + 1];
    for (unsigned x = b + 1; x < e; ++x) {  // insertion sort by column
      const unsigned v = cslot[x];
      const unsigned kv = (unsigned)(ckey[v] & 0xffffffffull);
      unsigned y = x;
      while (y > b && (unsigned)(ckey[cslot[y - 1]] & 0xffffffffull) > kv) {
        cslot[y] = cslot[y - 1];
        --y;
      }
      cslot[y] = v;
    }
    for (unsigned x = b; x < e; ++x) {
      const unsigned v = cslot[x];
      const unsigned long long kk = ckey[v];
      ci[x] = (int)(kk >> 32);
      cj[x] = (int)(kk & 0xffffffffull);
#pragma unroll
      for (int f = 0; f < 5; ++f) out[(int64_t)f * P + x] = cpay[f * cap + v];
    }
  }
  // loss-of-separation pairs of row r
  {
    const unsigned b = rowoff[nrows + 1 + r] - (unsigned)P, e = rowoff[nrows + 2 + r] - (unsigned)P;
    for (unsigned x = b + 1; x < e; ++x) {
      const unsigned v = lslot[x];
      const unsigned kv = (unsigned)(ckey[v] & 0xffffffffull);
      unsigned y = x;
      while (y > b && (unsigned)(ckey[lslot[y - 1]] & 0xffffffffull) > kv) {
        lslot[y] = lslot[y - 1];
        --y;
      }
      lslot[y] = v;
    }
    for (unsigned x = b; x < e; ++x) {
      const unsigned long long kk = ckey[lslot[x]];
      li[x] = (int)(kk >> 32);
      lj[x] = (int)(kk & 0xffffffffull);
    }
  }
}

// zero the per-detect state in one launch: counters (all but `tiles` unless
// full), the dequeue shards and the per-row outputs / counts
__global__ __launch_bounds__(256) void k_zero(int nrows, int full, Counters *__restrict__ cnt,
                                              unsigned long long *__restrict__ work,
                                              unsigned char *__restrict__ inconf,
                                              unsigned long long *__restrict__ tcpamax,
                                              unsigned *__restrict__ rowcnt) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k == 0) {
    const unsigned long long tiles = cnt->tiles;
    *cnt = Counters{};
    if (!full) cnt->tiles = tiles;
  }
  if (k < kWorkShards * kWorkStride) work[k] = 0;
  if (k < nrows) {
    inconf[k] = 0;
    tcpamax[k] = 0;
  }
  if (k < 2 * (nrows + 1)) rowcnt[k] = 0;
}

// ------------------------------------------------------------------ host side
static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }


// spatial sort of cnt positions starting at original index base -> perm
static int spatial_order(Ctx *c, int cnt, int base, const double *lat, const double *lon,
                         DevBuf &key, DevBuf &idx, DevBuf &key2, DevBuf &perm) {
  if (!ensure(c, key, (size_t)cnt * 4, "keys") || !ensure(c, idx, (size_t)cnt * 4, "key idx") ||
      !ensure(c, key2, (size_t)cnt * 4, "sorted keys") || !ensure(c, perm, (size_t)cnt * 4, "perm"))
    return -1;
  hipLaunchKernelGGL(k_keys, dim3(blocks_for(cnt, 256)), dim3(256), 0, c->stream, cnt, base, lat, lon,
                     (unsigned *)key.p, (unsigned *)idx.p);
  BSA_HIP(c, hipGetLastError());
  size_t tmp = 0;
  BSA_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (unsigned *)key.p, (unsigned *)key2.p,
                                                (unsigned *)idx.p, (unsigned *)perm.p, cnt, 0, 30,
                                                c->stream));
  if (!ensure(c, c->sort_tmp, std::max<size_t>(tmp, 16), "sort scratch")) return -1;
  tmp = c->sort_tmp.bytes;
  BSA_HIP(c, hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp, (unsigned *)key.p,
                                                (unsigned *)key2.p, (unsigned *)idx.p,
                                                (unsigned *)perm.p, cnt, 0, 30, c->stream));
  return 0;
}


int detect(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
           int64_t *n_conf, int64_t *n_los) {
  const int64_t n = c->n;
  if (re <= 0) re = n;
  if (rb < 0 || rb > re || re > n)
    return fail(c, "bad row range [%lld, %lld) for n=%lld", (long long)rb, (long long)re, (long long)n);
  if (n > (int64_t)0x7fffffff) return fail(c, "n=%lld exceeds 2^31-1", (long long)n);
  const int64_t nrows = re - rb;
  c->have_pairs = false;
  c->last_rb = rb;
  c->last_re = re;
  c->last_flags = flags;
  c->last_conf = c->last_los = c->last_cand = 0;
  if (!ensure(c, c->counters, sizeof(Counters), "counters") ||
      !ensure(c, c->inconf, (size_t)(nrows > 0 ? nrows : 1), "inconf") ||
      !ensure(c, c->tcpamax, (size_t)(nrows > 0 ? nrows : 1) * 8, "tcpamax") ||
      !ensure(c, c->workq, kWorkShards * kWorkStride * 8, "work counters") ||
      !ensure(c, c->rowcnt, (size_t)(2 * (nrows + 1)) * 4, "row counts") ||
      !ensure(c, c->rowoff, (size_t)(2 * (nrows + 1)) * 4, "row offsets"))
    return -1;
  BSA_HIP(c, hipEventRecord(c->ev[0], c->stream));
  Counters *dcnt = (Counters *)c->counters.p;
  auto zero = [&](int full) -> int {
    const int64_t m = std::max<int64_t>(2 * (nrows + 1), kWorkShards * kWorkStride);
    hipLaunchKernelGGL(k_zero, dim3(blocks_for(m, 256)), dim3(256), 0, c->stream, (int)nrows, full, dcnt,
                       (unsigned long long *)c->workq.p, (unsigned char *)c->inconf.p,
                       (unsigned long long *)c->tcpamax.p, (unsigned *)c->rowcnt.p);
    BSA_HIP(c, hipGetLastError());
    return 0;
  };
  if (zero(1)) return -1;
  if (n == 0 || nrows == 0) {
    for (int e = 1; e < 5; ++e) BSA_HIP(c, hipEventRecord(c->ev[e], c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    c->ev_valid = true;
    c->have_pairs = true;
    *n_conf = *n_los = 0;
    return 0;
  }
  const int noprune = (flags & BSA_FLAG_NOPRUNE) ? 1 : 0;
  const bool distinct = c->has_intruder;
  DevBuf *I = distinct ? c->intr : c->own;
  SoA6 own{(const double *)c->own[0].p, (const double *)c->own[1].p, (const double *)c->own[2].p,
           (const double *)c->own[3].p, (const double *)c->own[4].p, (const double *)c->own[5].p};
  SoA6 intr{(const double *)I[0].p, (const double *)I[1].p, (const double *)I[2].p,
            (const double *)I[3].p, (const double *)I[4].p, (const double *)I[5].p};

  // ---- K0a spatial order.  Any permutation gives identical results (the
  // output is re-sorted canonically), so the order is reused for up to
  // kResortEvery calls on the same shape: aircraft move ~km between calls,
  // tiles span ~100 km.  Rows share the column order when own == intruder
  // and the whole range is detected.
  const bool shared = !distinct && rb == 0 && re == n;
  const bool resort = !c->perm_valid || c->perm_n != n || c->perm_rb != rb || c->perm_re != re ||
                      c->perm_shared != shared || c->perm_distinct != distinct ||
                      (flags & BSA_FLAG_RESORT) || c->perm_age >= kResortEvery;
  if (resort) {
    if (spatial_order(c, (int)n, 0, intr.lat, intr.lon, c->key_c, c->idx_c, c->key_c2, c->perm_c)) return -1;
    if (!shared &&
        spatial_order(c, (int)nrows, (int)rb, own.lat, own.lon, c->key_r, c->idx_r, c->key_r2, c->perm_r))
      return -1;
    c->perm_valid = true;
    c->perm_n = n;
    c->perm_rb = rb;
    c->perm_re = re;
    c->perm_shared = shared;
    c->perm_distinct = distinct;
    c->perm_age = 0;
  }
  c->perm_age++;
  const unsigned *perm_r = (const unsigned *)(shared ? c->perm_c.p : c->perm_r.p);
  const unsigned *perm_c = (const unsigned *)c->perm_c.p;

  // ---- K0b records in sorted order
  if (!ensure(c, c->rowrec, nrows * sizeof(RowRec), "row records") ||
      !ensure(c, c->colrec, n * sizeof(ColRec), "column records") ||
      !ensure(c, c->pfrow, nrows * sizeof(PFRec), "prefilter rows") ||
      !ensure(c, c->pfcol, n * sizeof(PFRec), "prefilter columns") ||
      !ensure(c, c->pfauxrow, nrows * sizeof(PFAux), "prefilter row aux") ||
      !ensure(c, c->pfauxcol, n * sizeof(PFAux), "prefilter column aux"))
    return -1;
  hipLaunchKernelGGL(k_prep_rows, dim3(blocks_for(nrows, 256)), dim3(256), 0, c->stream, (int)nrows, perm_r,
                     own, intr, rpz, hpz, tla, (RowRec *)c->rowrec.p, (PFRec *)c->pfrow.p,
                     (PFAux *)c->pfauxrow.p);
  BSA_HIP(c, hipGetLastError());
  hipLaunchKernelGGL(k_prep_cols, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, (int)n, perm_c, own,
                     intr, distinct ? 1 : 0, rpz, hpz, tla, (ColRec *)c->colrec.p, (PFRec *)c->pfcol.p,
                     (PFAux *)c->pfauxcol.p);
  BSA_HIP(c, hipGetLastError());
  // ---- K0c/K0d group / tile boxes and the tile-pair work list
  const int nrt = (int)((nrows + kTile - 1) / kTile), nct = (int)((n + kTile - 1) / kTile);
  const long long ntp = (long long)nrt * nct;
  const int ngr = (int)((nrows + kGroup - 1) / kGroup), ngc = (int)((n + kGroup - 1) / kGroup);
  if (!ensure(c, c->tbox_r, nrt * sizeof(TileBox), "row tile boxes") ||
      !ensure(c, c->tbox_c, nct * sizeof(TileBox), "column tile boxes") ||
      !ensure(c, c->gbox_r, ngr * sizeof(TileBox), "row group boxes") ||
      !ensure(c, c->gbox_c, ngc * sizeof(TileBox), "column group boxes") ||
      !ensure(c, c->tilepairs, (size_t)ntp * sizeof(uint2), "tile pairs"))
    return -1;
  hipLaunchKernelGGL(k_groupbox, dim3(blocks_for(ngr, 4)), dim3(256), 0, c->stream, (int)nrows,
                     (const PFRec *)c->pfrow.p, (TileBox *)c->gbox_r.p);
  hipLaunchKernelGGL(k_groupbox, dim3(blocks_for(ngc, 4)), dim3(256), 0, c->stream, (int)n,
                     (const PFRec *)c->pfcol.p, (TileBox *)c->gbox_c.p);
  hipLaunchKernelGGL(k_tileunion, dim3(blocks_for(nrt, 256)), dim3(256), 0, c->stream, nrt, ngr,
                     (const TileBox *)c->gbox_r.p, (TileBox *)c->tbox_r.p);
  hipLaunchKernelGGL(k_tileunion, dim3(blocks_for(nct, 256)), dim3(256), 0, c->stream, nct, ngc,
                     (const TileBox *)c->gbox_c.p, (TileBox *)c->tbox_c.p);
  hipLaunchKernelGGL(k_tilepairs, dim3((unsigned)((ntp + 255) / 256)), dim3(256), 0, c->stream, nrt, nct,
                     (const TileBox *)c->tbox_r.p, (const TileBox *)c->tbox_c.p, noprune,
                     (uint2 *)c->tilepairs.p, &dcnt->tiles);
  BSA_HIP(c, hipGetLastError());
  BSA_HIP(c, hipEventRecord(c->ev[1], c->stream));

  if (c->cand_cap == 0) c->cand_cap = (unsigned long long)std::max<int64_t>(1 << 20, 16 * nrows);
  const float T = (float)(tla > 0.0 ? tla : 0.0);
  const float lim = (float)((rpz + kEABS) / (1.0 - kE1));
  const RefineParams rp{(float)rpz, (float)hpz, T, lim * lim};
  const int nscan = (int)(2 * (nrows + 1));
  size_t scan_tmp = 0;
  BSA_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp, (const unsigned *)c->rowcnt.p,
                                              (unsigned *)c->rowoff.p, nscan, c->stream));
  if (!ensure(c, c->sort_tmp, std::max<size_t>(scan_tmp, 16), "scan scratch")) return -1;
  Counters h;
  unsigned tot[2] = {0, 0};  // P and P + L from the scan
  for (int attempt = 0;; ++attempt) {
    const unsigned long long cap = c->cand_cap;
    if (!ensure(c, c->cand, cap * sizeof(uint2), "candidate pairs") ||
        !ensure(c, c->cflag, cap, "candidate flags") ||
        !ensure(c, c->ckey, cap * 8, "candidate keys") ||
        !ensure(c, c->cpay, cap * 5 * 8, "candidate payload"))
      return -1;
    if (attempt > 0 && zero(0)) return -1;
    // ---- K1a prefilter: persistent grid, 6 workgroups per CU (LDS/SGPR-limited
    // residency), at least one workgroup per dequeue shard
    const unsigned pf_grid =
        (unsigned)std::max<long long>(kWorkShards, std::min<long long>(ntp * PF_WAVES, 256 * 6));
    if (noprune)
      hipLaunchKernelGGL(k_prefilter<true>, dim3(pf_grid), dim3(PF_BLOCK), 0, c->stream,
                         (const PFRec *)c->pfrow.p, (const PFAux *)c->pfauxrow.p, (int)nrows,
                         (const PFRec *)c->pfcol.p, (const PFAux *)c->pfauxcol.p, (int)n,
                         (const TileBox *)c->gbox_r.p, (const TileBox *)c->gbox_c.p,
                         (const uint2 *)c->tilepairs.p, dcnt, (unsigned long long *)c->workq.p, rp,
                         (uint2 *)c->cand.p, cap);
    else
      hipLaunchKernelGGL(k_prefilter<false>, dim3(pf_grid), dim3(PF_BLOCK), 0, c->stream,
                         (const PFRec *)c->pfrow.p, (const PFAux *)c->pfauxrow.p, (int)nrows,
                         (const PFRec *)c->pfcol.p, (const PFAux *)c->pfauxcol.p, (int)n,
                         (const TileBox *)c->gbox_r.p, (const TileBox *)c->gbox_c.p,
                         (const uint2 *)c->tilepairs.p, dcnt, (unsigned long long *)c->workq.p, rp,
                         (uint2 *)c->cand.p, cap);
    BSA_HIP(c, hipGetLastError());
    BSA_HIP(c, hipEventRecord(c->ev[2], c->stream));
    // ---- K1b exact evaluation: grid-stride over the device-side count, one
    // resident round (4 workgroups per CU at its register budget)
    hipLaunchKernelGGL(k_exact, dim3(256 * 4), dim3(256), 0, c->stream, (const RowRec *)c->rowrec.p,
                       (const ColRec *)c->colrec.p, perm_r, perm_c, (const uint2 *)c->cand.p, &dcnt->cand,
                       cap, rpz, hpz, tla, (int)rb, (int)nrows, (unsigned char *)c->cflag.p,
                       (unsigned long long *)c->ckey.p, (double *)c->cpay.p, (unsigned char *)c->inconf.p,
                       (unsigned long long *)c->tcpamax.p, (unsigned *)c->rowcnt.p);
    BSA_HIP(c, hipGetLastError());
    // ---- K2 part 1: row offsets (exclusive scan of [conf per row | 0 | LoS per row | 0])
    size_t tmp = c->sort_tmp.bytes;
    BSA_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->sort_tmp.p, tmp, (const unsigned *)c->rowcnt.p,
                                                (unsigned *)c->rowoff.p, nscan, c->stream));
    BSA_HIP(c, hipEventRecord(c->ev[3], c->stream));
    // the detect's only host sync: candidate count + totals P and P + L
    BSA_HIP(c, hipMemcpyAsync(&h, c->counters.p, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipMemcpyAsync(&tot[0], (const unsigned *)c->rowoff.p + nrows, 4, hipMemcpyDeviceToHost,
                              c->stream));
    BSA_HIP(c, hipMemcpyAsync(&tot[1], (const unsigned *)c->rowoff.p + nscan - 1, 4,
                              hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    if (h.cand <= cap) break;
    if (attempt > 3) return fail(c, "candidate buffer overflow (%llu)", h.cand);
    c->cand_cap = h.cand + h.cand / 4 + 1024;
  }
  c->last_cand = (int64_t)h.cand;
  c->last_tiles = (int64_t)h.tiles;
  c->last_tiles_total = ntp;
  c->last_groups = (int64_t)h.groups;

  // ---- K2 part 2: scatter into row segments, per-row insertion sort + gather
  const int64_t P = (int64_t)tot[0], L = (int64_t)tot[1] - (int64_t)tot[0];
  if (!ensure(c, c->cval2, (size_t)std::max<int64_t>(P, 1) * 4, "conflict slots") ||
      !ensure(c, c->lslot, (size_t)std::max<int64_t>(L, 1) * 4, "los slots") ||
      !ensure(c, c->out_ci, (size_t)std::max<int64_t>(P, 1) * 4, "ci") ||
      !ensure(c, c->out_cj, (size_t)std::max<int64_t>(P, 1) * 4, "cj") ||
      !ensure(c, c->out_pay, (size_t)std::max<int64_t>(P, 1) * 5 * 8, "conflict outputs") ||
      !ensure(c, c->out_li, (size_t)std::max<int64_t>(L, 1) * 4, "li") ||
      !ensure(c, c->out_lj, (size_t)std::max<int64_t>(L, 1) * 4, "lj"))
    return -1;
  if (P + L > 0) {
    hipLaunchKernelGGL(k_scatter, dim3(256 * 4), dim3(256), 0, c->stream, &dcnt->cand, c->cand_cap,
                       (int)rb, (int)nrows, (const unsigned char *)c->cflag.p,
                       (const unsigned long long *)c->ckey.p, (const unsigned *)c->rowoff.p,
                       (unsigned *)c->rowcnt.p, (unsigned *)c->cval2.p, (unsigned *)c->lslot.p);
    BSA_HIP(c, hipGetLastError());
    hipLaunchKernelGGL(k_rowsort, dim3(blocks_for(nrows, 256)), dim3(256), 0, c->stream, (int)nrows, P,
                       (const unsigned *)c->rowoff.p, (const unsigned long long *)c->ckey.p,
                       (unsigned *)c->cval2.p, (const double *)c->cpay.p, c->cand_cap,
                       (unsigned *)c->lslot.p, (int *)c->out_ci.p, (int *)c->out_cj.p,
                       (double *)c->out_pay.p, (int *)c->out_li.p, (int *)c->out_lj.p);
    BSA_HIP(c, hipGetLastError());
  }
  BSA_HIP(c, hipEventRecord(c->ev[4], c->stream));
  c->ev_valid = true;
  c->last_conf = P;
  c->last_los = L;
  c->have_pairs = true;
  *n_conf = P;
  *n_los = L;
  return 0;
}

}  // namespace bsa
