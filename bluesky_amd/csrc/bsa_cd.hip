// K0 prep, K1a prefilter, K1b exact pair evaluation, K2 canonical sort.
//
// StateBasedCD.detect (bluesky/traffic/asas/StateBasedCD.py:7-103) with
// geo.qdrdist_matrix (bluesky/tools/geo.py:110-162) fused in, for gfx950.
//
// Structure:
//   K0 prep        one thread per aircraft: per-index fp64 records (the
//                  per-aircraft factors of the reference's N x N broadcasts)
//                  and fp32 prefilter records.
//   K1a prefilter  N-body tiled sweep over all (i, j): lane = ownship row
//                  (2 rows per lane), intruder tiles in LDS, broadcast reads.
//                  A conservative fp32 bound keeps every pair that could be a
//                  conflict or a loss of separation (proof in DESIGN.md);
//                  survivors are compacted through a per-wave LDS queue with
//                  ballot/mbcnt and one atomic per flush.
//   K1b exact      one lane per candidate: the reference's fp64 expression
//                  sequence, op for op (-ffp-contract=off), conflict / LoS
//                  outputs appended with one atomic per wave.
//   K2 sort        hipcub radix sort on key = (i << 32 | j), i.e. the
//                  reference's row-major np.where order, then a gather.
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

// ------------------------------------------------------------------ K0 prep
__device__ __forceinline__ float reach_h(double rpz, double gs, double tlap) {
  // horizontal half-bound in unit-sphere chord units: the pair keeps iff
  // chord < s_i + s_j, s = ((R/2 + (|gs| + 0.5e-3) tla)(1 + 1e-5)) / 6.3e6 + 1e-6
  double s = ((0.5 * rpz + (fabs(gs) + 0.5e-3) * tlap) * (1.0 + 1e-5)) / 6.3e6 + 1e-6;
  return isfinite(s) ? (float)s : INFINITY;
}
__device__ __forceinline__ float reach_v(double hpz, double vs, double alt, double tlap) {
  double h = (0.5 * hpz + (fabs(vs) + 0.5e-6) * tlap) * (1.0 + 1e-5) + 0.5 + 1e-6 * fabs(alt);
  return isfinite(h) ? (float)h : INFINITY;
}

__global__ __launch_bounds__(256) void k_prep(
    int n, const double *__restrict__ olat, const double *__restrict__ olon,
    const double *__restrict__ otrk, const double *__restrict__ ogs,
    const double *__restrict__ oalt, const double *__restrict__ ovs,
    const double *__restrict__ ilat, const double *__restrict__ ilon,
    const double *__restrict__ itrk, const double *__restrict__ igs,
    const double *__restrict__ ialt, const double *__restrict__ ivs, int distinct,
    double rpz, double hpz, double tla, RowRec *__restrict__ R, ColRec *__restrict__ C,
    PFRec *__restrict__ PR, PFRec *__restrict__ PC) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double a = kWGS84_A;
  const double tlap = tla > 0.0 ? tla : 0.0;

  // ownship k: row geometry, column velocity
  const double la_o = olat[k], lo_o = olon[k];
  const double rad_o = la_o * kD2R;
  const double sin_o = sin(rad_o), cos_o = cos(rad_o);
  const double trk_o = otrk[k] * kD2R;
  const double u_o = ogs[k] * sin(trk_o), v_o = ogs[k] * cos(trk_o);
  // intruder k: column geometry, row velocity
  double la_i = la_o, lo_i = lo_o, sin_i = sin_o, cos_i = cos_o, u_i = u_o, v_i = v_o;
  double alt_i = oalt[k], vs_i = ovs[k], gs_i = ogs[k];
  if (distinct) {
    la_i = ilat[k];
    lo_i = ilon[k];
    const double rad_i = la_i * kD2R;
    sin_i = sin(rad_i);
    cos_i = cos(rad_i);
    const double trk_i = itrk[k] * kD2R;
    gs_i = igs[k];
    u_i = gs_i * sin(trk_i);
    v_i = gs_i * cos(trk_i);
    alt_i = ialt[k];
    vs_i = ivs[k];
  }

  RowRec r;
  r.lat = la_o;
  r.lon = lo_o;
  r.sinlat = sin_o;
  r.coslat = cos_o;
  r.hemA = fabs(la_o) * (rwgs84(la_o) + a);
  r.u = u_i;
  r.v = v_i;
  r.alt = alt_i;
  r.vs = vs_i;
  for (int q = 0; q < 7; ++q) r.pad[q] = 0.0;
  R[k] = r;

  ColRec c;
  c.lat = la_i;
  c.lon = lo_i;
  c.sinlat = sin_i;
  c.coslat = cos_i;
  c.hemA = distinct ? fabs(la_i) * (rwgs84(la_i) + a) : r.hemA;
  c.u = u_o;
  c.v = v_o;
  c.alt = oalt[k];
  c.vs = ovs[k];
  c.eps = (la_o == 0.0) ? 0.000001 : 0.0;
  for (int q = 0; q < 6; ++q) c.pad[q] = 0.0;
  C[k] = c;

  // fp32 prefilter records (accuracy is covered by the margins in reach_*)
  PFRec pr, pc;
  const double lon_or = lo_o * kD2R, lon_ir = lo_i * kD2R;
  pr.x = (float)(cos_o * cos(lon_or));
  pr.y = (float)(cos_o * sin(lon_or));
  pr.z = (float)sin_o;
  pr.s = reach_h(rpz, gs_i, tlap);
  pr.alt = (float)alt_i;
  pr.h = reach_v(hpz, vs_i, alt_i, tlap);
  pr.pad0 = pr.pad1 = 0.f;
  pc.x = (float)(cos_i * cos(lon_ir));
  pc.y = (float)(cos_i * sin(lon_ir));
  pc.z = (float)sin_i;
  // (own.lat[j] == 0) makes the different-hemisphere radius unbounded below
  // when own != intruder (geo.py:128): never prune such a column.
  pc.s = (distinct && la_o == 0.0) ? INFINITY : reach_h(rpz, ogs[k], tlap);
  pc.alt = (float)oalt[k];
  pc.h = reach_v(hpz, ovs[k], oalt[k], tlap);
  pc.pad0 = pc.pad1 = 0.f;
  if (!(isfinite(pr.x) && isfinite(pr.y) && isfinite(pr.z))) pr.s = INFINITY;
  if (!(isfinite(pc.x) && isfinite(pc.y) && isfinite(pc.z))) pc.s = INFINITY;
  PR[k] = pr;
  PC[k] = pc;
}

// ------------------------------------------------------------------ K1a prefilter
constexpr int PF_BLOCK = 256;
constexpr int PF_RPT = 2;                    // ownship rows per lane
constexpr int PF_ROWS = PF_BLOCK * PF_RPT;   // rows per workgroup
constexpr int PF_TILE = 512;                 // intruder columns per LDS tile (16 KiB)
constexpr int PF_QCAP = 1024;                // per-wave candidate queue (8 KiB)
constexpr int PF_WAVES = PF_BLOCK / 64;

__device__ __forceinline__ unsigned lane_prefix(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

__device__ __forceinline__ unsigned long long wave_bcast_u64(unsigned long long v) {
  unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ bool pf_keep(const PFRec &a, const PFRec &c) {
  const float dx = c.x - a.x, dy = c.y - a.y, dz = c.z - a.z;
  const float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
  const float st = a.s + c.s;
  const float dh = __builtin_fabsf(c.alt - a.alt);
  return (d2 < st * st) & (dh < a.h + c.h);
}

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

__global__ __launch_bounds__(PF_BLOCK) void k_prefilter(
    const PFRec *__restrict__ prow, const PFRec *__restrict__ pcol, int rb, int re, int ncols,
    int cols_per_split, int noprune, uint2 *__restrict__ cand,
    unsigned long long *__restrict__ cand_count, unsigned long long cap) {
  __shared__ PFRec tile[PF_TILE];
  __shared__ uint2 queue[PF_WAVES][PF_QCAP];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int r0 = rb + blockIdx.x * PF_ROWS + tid;
  const int r1 = r0 + PF_BLOCK;
  PFRec a, b;
  const float qnan = __builtin_nanf("");
  if (r0 < re) a = prow[r0]; else { a.x = a.y = a.z = qnan; a.s = a.alt = a.h = 0.f; }
  if (r1 < re) b = prow[r1]; else { b.x = b.y = b.z = qnan; b.s = b.alt = b.h = 0.f; }
  const bool va = r0 < re, vb = r1 < re;
  const int c0 = blockIdx.y * cols_per_split;
  const int c1 = min(ncols, c0 + cols_per_split);
  uint2 *q = queue[w];
  unsigned qn = 0;  // wave-uniform queue fill
  for (int t0 = c0; t0 < c1; t0 += PF_TILE) {
    const int nt = min(PF_TILE, c1 - t0);
    __syncthreads();
    for (int k = tid; k < nt; k += PF_BLOCK) tile[k] = pcol[t0 + k];
    __syncthreads();
    for (int jj = 0; jj < nt; ++jj) {
      const PFRec c = tile[jj];
      const bool ka = noprune ? va : pf_keep(a, c);
      const bool kb = noprune ? vb : pf_keep(b, c);
      const unsigned long long ma = __ballot(ka), mb = __ballot(kb);
      if (ma | mb) {
        const unsigned j = (unsigned)(t0 + jj);
        if (ka) q[qn + lane_prefix(ma)] = make_uint2((unsigned)r0, j);
        qn += (unsigned)__popcll(ma);
        if (kb) q[qn + lane_prefix(mb)] = make_uint2((unsigned)r1, j);
        qn += (unsigned)__popcll(mb);
        if (qn > (unsigned)(PF_QCAP - 2 * 64)) {
          pf_flush(q, qn, lane, cand, cand_count, cap);
          qn = 0;
        }
      }
    }
  }
  if (qn) pf_flush(q, qn, lane, cand, cand_count, cap);
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

__global__ __launch_bounds__(256) void k_exact(
    const RowRec *__restrict__ R, const ColRec *__restrict__ C, const uint2 *__restrict__ cand,
    unsigned long long ncand, double rpz, double hpz, double tla, int rb,
    unsigned long long *__restrict__ ckey, unsigned *__restrict__ cval,
    double *__restrict__ cpay, unsigned long long conf_cap,
    unsigned long long *__restrict__ lkey, unsigned long long los_cap,
    Counters *__restrict__ cnt, unsigned char *__restrict__ inconf,
    unsigned long long *__restrict__ tcpamax_bits) {
  const int lane = threadIdx.x & 63;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long idx = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
       idx < ncand; idx += stride) {
    const uint2 p = cand[idx];
    bool conf = false, los = false;
    PairResult o;
    if (p.x != p.y) {
      o = eval_pair(R[p.x], C[p.y], rpz, hpz, tla);
      conf = o.conf;
      los = o.los;
    }
    const unsigned long long key = ((unsigned long long)p.x << 32) | p.y;
    const unsigned long long mc = __ballot(conf);
    if (mc) {
      const int leader = __builtin_ctzll(mc);
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&cnt->conf, (unsigned long long)__popcll(mc));
      base = __shfl(base, leader);
      if (conf) {
        const unsigned long long slot = base + lane_prefix(mc);
        if (slot < conf_cap) {
          ckey[slot] = key;
          cval[slot] = (unsigned)slot;
          cpay[0 * conf_cap + slot] = o.qdr;
          cpay[1 * conf_cap + slot] = o.dist;
          cpay[2 * conf_cap + slot] = o.tcpa;
          cpay[3 * conf_cap + slot] = o.tin;
          cpay[4 * conf_cap + slot] = o.dcpa;
        }
        const int row = (int)p.x - rb;
        inconf[row] = 1;
        // tcpamax = max_j(tcpa * swconfl) >= +-0 (StateBasedCD.py:90): only
        // positive tcpa can raise it, and positive doubles order as integers.
        if (o.tcpa > 0.0) atomicMax(&tcpamax_bits[row], (unsigned long long)__double_as_longlong(o.tcpa));
      }
    }
    const unsigned long long ml = __ballot(los);
    if (ml) {
      const int leader = __builtin_ctzll(ml);
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&cnt->los, (unsigned long long)__popcll(ml));
      base = __shfl(base, leader);
      if (los) {
        const unsigned long long slot = base + lane_prefix(ml);
        if (slot < los_cap) lkey[slot] = key;
      }
    }
  }
}

// ------------------------------------------------------------------ K2 gather
__global__ __launch_bounds__(256) void k_gather_conf(
    int64_t P, const unsigned long long *__restrict__ key, const unsigned *__restrict__ val,
    const double *__restrict__ pay, unsigned long long cap, int *__restrict__ ci,
    int *__restrict__ cj, double *__restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= P) return;
  const unsigned long long kk = key[k];
  const unsigned s = val[k];
  ci[k] = (int)(kk >> 32);
  cj[k] = (int)(kk & 0xffffffffull);
#pragma unroll
  for (int f = 0; f < 5; ++f) out[f * P + k] = pay[f * cap + s];
}

__global__ __launch_bounds__(256) void k_split_los(int64_t L, const unsigned long long *__restrict__ key,
                                                   int *__restrict__ li, int *__restrict__ lj) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= L) return;
  const unsigned long long kk = key[k];
  li[k] = (int)(kk >> 32);
  lj[k] = (int)(kk & 0xffffffffull);
}

// ------------------------------------------------------------------ host side
static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

int prep_records(Ctx *c, double rpz, double hpz, double tla) {
  const int64_t n = c->n;
  if (!ensure(c, c->rowrec, n * sizeof(RowRec), "row records") ||
      !ensure(c, c->colrec, n * sizeof(ColRec), "column records") ||
      !ensure(c, c->pfrow, n * sizeof(PFRec), "prefilter rows") ||
      !ensure(c, c->pfcol, n * sizeof(PFRec), "prefilter columns"))
    return -1;
  DevBuf *I = c->has_intruder ? c->intr : c->own;
  hipLaunchKernelGGL(k_prep, dim3(blocks_for(n, 256)), dim3(256), 0, c->stream, (int)n,
                     (const double *)c->own[0].p, (const double *)c->own[1].p,
                     (const double *)c->own[2].p, (const double *)c->own[3].p,
                     (const double *)c->own[4].p, (const double *)c->own[5].p,
                     (const double *)I[0].p, (const double *)I[1].p, (const double *)I[2].p,
                     (const double *)I[3].p, (const double *)I[4].p, (const double *)I[5].p,
                     c->has_intruder ? 1 : 0, rpz, hpz, tla, (RowRec *)c->rowrec.p,
                     (ColRec *)c->colrec.p, (PFRec *)c->pfrow.p, (PFRec *)c->pfcol.p);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

static int read_counters(Ctx *c, Counters *h) {
  BSA_HIP(c, hipMemcpyAsync(h, c->counters.p, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int bitwidth(int64_t n) {
  int b = 1;
  while ((int64_t(1) << b) < n) ++b;
  return b;
}

int detect(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
           int64_t *n_conf, int64_t *n_los) {
  const int64_t n = c->n;
  if (re <= 0) re = n;
  if (rb < 0 || rb > re || re > n) return fail(c, "bad row range [%lld, %lld) for n=%lld",
                                                 (long long)rb, (long long)re, (long long)n);
  if (n > (int64_t)0x7fffffff) return fail(c, "n=%lld exceeds 2^31-1", (long long)n);
  const int64_t nrows = re - rb;
  c->have_pairs = false;
  c->last_rb = rb;
  c->last_re = re;
  c->last_flags = flags;
  c->last_conf = c->last_los = c->last_cand = 0;
  if (!ensure(c, c->counters, sizeof(Counters), "counters") ||
      !ensure(c, c->inconf, (size_t)(nrows > 0 ? nrows : 1), "inconf") ||
      !ensure(c, c->tcpamax, (size_t)(nrows > 0 ? nrows : 1) * 8, "tcpamax"))
    return -1;
  BSA_HIP(c, hipEventRecord(c->ev[0], c->stream));
  if (n == 0 || nrows == 0) {
    for (int e = 1; e < 5; ++e) BSA_HIP(c, hipEventRecord(c->ev[e], c->stream));
    c->ev_valid = true;
    c->have_pairs = true;
    *n_conf = *n_los = 0;
    return 0;
  }
  if (prep_records(c, rpz, hpz, tla)) return -1;
  BSA_HIP(c, hipEventRecord(c->ev[1], c->stream));

  // ---- K1a prefilter (retry with a larger candidate buffer on overflow)
  if (c->cand_cap == 0) c->cand_cap = (unsigned long long)std::max<int64_t>(1 << 20, 64 * nrows);
  const int noprune = (flags & BSA_FLAG_NOPRUNE) ? 1 : 0;
  const unsigned rowblocks = blocks_for(nrows, PF_ROWS);
  unsigned splits = (unsigned)std::max<int64_t>(1, (4096 + rowblocks - 1) / rowblocks);
  splits = (unsigned)std::min<int64_t>(splits, std::max<int64_t>(1, n / PF_TILE));
  const int cols_per_split = (int)((n + splits - 1) / splits);
  Counters h;
  for (int attempt = 0;; ++attempt) {
    if (!ensure(c, c->cand, c->cand_cap * sizeof(uint2), "candidate pairs")) return -1;
    BSA_HIP(c, hipMemsetAsync(c->counters.p, 0, sizeof(Counters), c->stream));
    hipLaunchKernelGGL(k_prefilter, dim3(rowblocks, splits), dim3(PF_BLOCK), 0, c->stream,
                       (const PFRec *)c->pfrow.p, (const PFRec *)c->pfcol.p, (int)rb, (int)re,
                       (int)n, cols_per_split, noprune, (uint2 *)c->cand.p,
                       &((Counters *)c->counters.p)->cand, c->cand_cap);
    BSA_HIP(c, hipGetLastError());
    if (read_counters(c, &h)) return -1;
    if (h.cand <= c->cand_cap) break;
    if (attempt > 3) return fail(c, "candidate buffer overflow (%llu)", h.cand);
    c->cand_cap = h.cand + h.cand / 4 + 1024;
  }
  BSA_HIP(c, hipEventRecord(c->ev[2], c->stream));
  c->last_cand = (int64_t)h.cand;

  // ---- K1b exact evaluation (retry with larger outputs on overflow)
  if (c->conf_cap == 0) c->conf_cap = (unsigned long long)std::max<int64_t>(1 << 16, 8 * nrows);
  if (c->los_cap == 0) c->los_cap = (unsigned long long)std::max<int64_t>(1 << 16, 4 * nrows);
  const unsigned long long ncand = h.cand;
  for (int attempt = 0;; ++attempt) {
    if (!ensure(c, c->ckey, c->conf_cap * 8, "conflict keys") ||
        !ensure(c, c->cval, c->conf_cap * 4, "conflict slots") ||
        !ensure(c, c->cpay, c->conf_cap * 5 * 8, "conflict payload") ||
        !ensure(c, c->lkey, c->los_cap * 8, "los keys"))
      return -1;
    BSA_HIP(c, hipMemsetAsync(&((Counters *)c->counters.p)->conf, 0, 16, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->inconf.p, 0, nrows, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->tcpamax.p, 0, nrows * 8, c->stream));
    if (ncand) {
      const unsigned grid = (unsigned)std::min<unsigned long long>((ncand + 255) / 256, 1u << 16);
      hipLaunchKernelGGL(k_exact, dim3(grid), dim3(256), 0, c->stream, (const RowRec *)c->rowrec.p,
                         (const ColRec *)c->colrec.p, (const uint2 *)c->cand.p, ncand, rpz, hpz, tla,
                         (int)rb, (unsigned long long *)c->ckey.p, (unsigned *)c->cval.p,
                         (double *)c->cpay.p, c->conf_cap, (unsigned long long *)c->lkey.p,
                         c->los_cap, (Counters *)c->counters.p, (unsigned char *)c->inconf.p,
                         (unsigned long long *)c->tcpamax.p);
      BSA_HIP(c, hipGetLastError());
    }
    if (read_counters(c, &h)) return -1;
    if (h.conf <= c->conf_cap && h.los <= c->los_cap) break;
    if (attempt > 3) return fail(c, "pair buffer overflow (conf %llu, los %llu)", h.conf, h.los);
    if (h.conf > c->conf_cap) c->conf_cap = h.conf + h.conf / 4 + 1024;
    if (h.los > c->los_cap) c->los_cap = h.los + h.los / 4 + 1024;
  }
  BSA_HIP(c, hipEventRecord(c->ev[3], c->stream));

  // ---- K2 canonical row-major order
  const int64_t P = (int64_t)h.conf, L = (int64_t)h.los;
  const int end_bit = 32 + bitwidth(n);
  if (!ensure(c, c->ckey2, (size_t)std::max<int64_t>(P, 1) * 8, "sorted conflict keys") ||
      !ensure(c, c->cval2, (size_t)std::max<int64_t>(P, 1) * 4, "sorted conflict slots") ||
      !ensure(c, c->lkey2, (size_t)std::max<int64_t>(L, 1) * 8, "sorted los keys") ||
      !ensure(c, c->out_ci, (size_t)std::max<int64_t>(P, 1) * 4, "ci") ||
      !ensure(c, c->out_cj, (size_t)std::max<int64_t>(P, 1) * 4, "cj") ||
      !ensure(c, c->out_pay, (size_t)std::max<int64_t>(P, 1) * 5 * 8, "conflict outputs") ||
      !ensure(c, c->out_li, (size_t)std::max<int64_t>(L, 1) * 4, "li") ||
      !ensure(c, c->out_lj, (size_t)std::max<int64_t>(L, 1) * 4, "lj"))
    return -1;
  size_t t1 = 0, t2 = 0;
  BSA_HIP(c, hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (unsigned long long *)nullptr,
                                                (unsigned long long *)nullptr, (unsigned *)nullptr,
                                                (unsigned *)nullptr, (int)std::max<int64_t>(P, 1), 0,
                                                end_bit, c->stream));
  BSA_HIP(c, hipcub::DeviceRadixSort::SortKeys(nullptr, t2, (unsigned long long *)nullptr,
                                               (unsigned long long *)nullptr,
                                               (int)std::max<int64_t>(L, 1), 0, end_bit, c->stream));
  size_t tmp = std::max(t1, t2);
  if (!ensure(c, c->sort_tmp, std::max<size_t>(tmp, 16), "sort scratch")) return -1;
  if (P > 0) {
    BSA_HIP(c, hipcub::DeviceRadixSort::SortPairs(c->sort_tmp.p, tmp, (unsigned long long *)c->ckey.p,
                                                  (unsigned long long *)c->ckey2.p, (unsigned *)c->cval.p,
                                                  (unsigned *)c->cval2.p, (int)P, 0, end_bit, c->stream));
    hipLaunchKernelGGL(k_gather_conf, dim3(blocks_for(P, 256)), dim3(256), 0, c->stream, P,
                       (const unsigned long long *)c->ckey2.p, (const unsigned *)c->cval2.p,
                       (const double *)c->cpay.p, c->conf_cap, (int *)c->out_ci.p,
                       (int *)c->out_cj.p, (double *)c->out_pay.p);
    BSA_HIP(c, hipGetLastError());
  }
  if (L > 0) {
    tmp = std::max(t1, t2);
    BSA_HIP(c, hipcub::DeviceRadixSort::SortKeys(c->sort_tmp.p, tmp, (unsigned long long *)c->lkey.p,
                                                 (unsigned long long *)c->lkey2.p, (int)L, 0, end_bit,
                                                 c->stream));
    hipLaunchKernelGGL(k_split_los, dim3(blocks_for(L, 256)), dim3(256), 0, c->stream, L,
                       (const unsigned long long *)c->lkey2.p, (int *)c->out_li.p, (int *)c->out_lj.p);
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
