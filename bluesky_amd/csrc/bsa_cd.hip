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

#include <chrono>
#include <thread>

#include "bsa_box.h"
#include "bsa_geo_math.h"
#include "bsa_halo.h"
#include "bsa_internal.h"
#include "bsa_mvp_math.h"
#include "bsa_mvp_row.h"
#include "bsa_prep.h"
#include "bsa_sim_row.h"

#pragma clang fp contract(off)

namespace bsa {

// math helpers (np_max / np_min / np_rem / rwgs84) and the qdrdist entries: bsa_geo_math.h

// ------------------------------------------------------------------ K0a keys
__device__ __forceinline__ unsigned expand10(unsigned v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}
// Spatial order key: 3-D Hilbert index (10 bits per axis, Skilling's
// transpose form) of the unit position vector.  Consecutive keys are always
// adjacent cells (no Z-order jumps), so the 64-row groups and 8-column
// sub-groups cut from the sorted order have tighter boxes: ~15% fewer stage-1
// pair tests than Morton order at the 100k box (tools/cull_sim.py).  Any order
// gives identical results; only the culling efficiency depends on it.
__device__ __forceinline__ unsigned curve_key(const double p[3]) {
  unsigned X[3];
  for (int k = 0; k < 3; ++k) {
    if (!(p[k] == p[k]) || isinf(p[k])) return 0xffffffffu;
    int q = (int)((p[k] + 1.0) * 512.0);
    X[k] = (unsigned)(q < 0 ? 0 : (q > 1023 ? 1023 : q));
  }
  // axes -> transposed Hilbert index
  for (unsigned Q = 1u << 9; Q > 1u; Q >>= 1) {
    const unsigned P = Q - 1u;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const unsigned t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  unsigned t = 0;
  for (unsigned Q = 1u << 9; Q > 1u; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1u;
  X[0] ^= t;
  X[1] ^= t;
  X[2] ^= t;
  return (expand10(X[0]) << 2) | (expand10(X[1]) << 1) | expand10(X[2]);
}

// f > 0 (midpoint stage 1): key of the stage-1 point m = p + f (u e + v n)
// (make_pf_mid), so that sorted groups stay compact around the points the
// boxes bound; any order gives identical results
__global__ __launch_bounds__(256) void k_keys(int cnt, int base, const double *__restrict__ lat,
                                              const double *__restrict__ lon, const double *__restrict__ trk,
                                              const double *__restrict__ gs, double f,
                                              unsigned *__restrict__ key,
                                              unsigned *__restrict__ idx) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const int o = base + k;
  const double la = lat[o] * kD2R, lo = lon[o] * kD2R;
  double cl, sl, co, so;
  sincos(la, &sl, &cl);
  sincos(lo, &so, &co);
  double p[3] = {cl * co, cl * so, sl};
  if (f > 0.0) {
    const double t = trk[o] * kD2R, g = gs[o];
    double st, ct;
    sincos(t, &st, &ct);
    const double u = g * st, v = g * ct;
    const double m[3] = {p[0] + f * (-u * so - v * sl * co), p[1] + f * (u * co - v * sl * so), p[2] + f * (v * cl)};
    if (isfinite(m[0]) && isfinite(m[1]) && isfinite(m[2]))
      for (int q = 0; q < 3; ++q) p[q] = m[q];
  }
  key[k] = curve_key(p);
  idx[k] = (unsigned)o;
}

// Row records, sorted position k -> original row perm[k]: own[i] geometry,
// intruder[i] velocity / altitude (StateBasedCD.py:39-40,65-69 orientation).
__global__ __launch_bounds__(256) void k_prep_rows(int cnt, const unsigned *__restrict__ perm,
                                                   SoA6 own, SoA6 intr, double rpz, double hpz,
                                                   double tla, RowRec *__restrict__ R,
                                                   PFRec *__restrict__ PR, PFVel *__restrict__ PV,
                                                   float4 *__restrict__ PP, int mid, uint8_t *__restrict__ rowbad,
                                                   int rb) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const int o = (int)perm[k];
  const double tlap = tla > 0.0 ? tla : 0.0;
  const double la = own.lat[o], lo = own.lon[o];
  const double rad = la * kD2R;
  double sinl, cosl;
  sincos(rad, &sinl, &cosl);
  const double trk = intr.trk[o] * kD2R;
  const double gs = intr.gs[o];
  RowRec r;
  r.lat = la;
  r.lon = lo;
  r.sinlat = sinl;
  r.coslat = cosl;
  r.hemA = fabs(la) * (rwgs84_sc(sinl, cosl) + kWGS84_A);  // geo.py:127
  double st, ct;
  sincos(trk, &st, &ct);
  r.u = gs * st;                                 // StateBasedCD.py:36-37
  r.v = gs * ct;
  r.alt = intr.alt[o];
  r.vs = intr.vs[o];
  r.pad0 = 0.0;
  r.ilat = intr.lat[o];
  for (int q = 0; q < 5; ++q) r.pad[q] = 0.0;
  R[k] = r;
  const double lor = lo * kD2R;
  double coslo, sinlo;
  sincos(lor, &sinlo, &coslo);
  const double px = cosl * coslo, py = cosl * sinlo, pz = sinl;
  const PFRec p = mid ? make_pf_mid(px, py, pz, sinl, cosl, coslo, sinlo, r.u, r.v, gs, r.alt, r.vs, rpz, hpz, tlap)
                      : make_pf(px, py, pz, reach_h(rpz, gs, tlap), r.alt, reach_v(hpz, r.vs, r.alt, tlap));
  PP[k] = make_float4((float)px, (float)py, (float)pz, 0.f);
  PFVel v;
  v.u = (float)r.u;
  v.v = (float)r.v;
  v.vs = (float)r.vs;
  // within ~0.6 deg of a pole (or |lat| > 90: the refine's local east / north
  // basis is ill-conditioned), or a non-finite position: never refine
  v.flags = (!(cosl > 1e-2) || !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) ? 1u : 0u;
  // every tcpa of the row, hence its tcpamax, is NaN (K2; rows in index order)
  rowbad[o - rb] = (isfinite(la) && isfinite(lo) && isfinite(r.u) && isfinite(r.v)) ? 0 : 1;
  PR[k] = p;
  PV[k] = v;
}

// Candidate-list reuse.  A list built with every aircraft's
// reach inflated by its budgets (horizontal sh, vertical sv) stays a superset
// of the exact list while every aircraft's drift since the build stays inside
// them: drift_h = |dchord| * kRS * L + |dvel| * T, drift_v = |dalt| + |dvs| * T
// (L bounds the rotation of the refine's local basis, chord <= kRefineChord).
struct ReuseParams {
  const Snap *build;  // snapshot of the last build (nullptr: reuse off)
  Snap *cur;          // this detect's state (becomes the snapshot on a build)
  unsigned *ctl;      // [0] build flag (set here on a budget overrun), [1] detects since build
  float *use;         // per wave: largest horizontal / vertical budget fraction used
  float sh_chord;     // horizontal budget in chord units (added to the stage-1 reach)
  double sh;          // horizontal budget [m, refine units]
  double sv_default, sv_min, sv_max, ktarget;
  int valid;          // the snapshot belongs to this perm / parameters
};
constexpr double kRefineChord = 0.03;  // the refine keeps (without refining) pairs with a longer chord

constexpr int kWorkShards = 32;  // dequeue counters (4 per XCD group): a returning atomic on one
                                 // word saturates at ~88 dequeues/us (MI355X_MICROARCH 'dequeue')
constexpr int kWorkStride = 16;  // u64 words between counters (128 B apart)

// K2 with row buckets (k_rank_rows): one workgroup per kRankRows rows; the
// pair counts of every block (k_rowblk) follow the 2 (nrows + 1) per-row
// counts, so the row offsets need no scan with a look-back chain.  (K1b
// counting them with atomics, one per wave and block, cost 12 us at the 100k
// box: the per-block words were hit by every wave of a block's rows at once.)
#ifndef BSA_RANK_ROWS
#define BSA_RANK_ROWS 512
#endif
constexpr int kRankRows = BSA_RANK_ROWS;
static_assert(kRankRows % 64 == 0 && kRankRows <= 1024, "whole waves per K2 block");
constexpr int kRankLds = 3 * kRankRows;  // pairs per block folded from LDS (512 rows: 67 KB, 2 blocks per CU)
// lanes per workgroup of k_rank_rows: its rows take one lane each, its pairs
// (~1.7 per row at the 100k box) one lane each.  Two lanes per row place a
// block's pairs in one pass instead of two, but the 1024-lane workgroup caps
// the kernel at 128 VGPRs (7 spilled): K2 27.7 -> 29.0 us at the 100k box
// (A/B on one box, round 4), so one
#ifndef BSA_RANK_LANES_PER_ROW
#define BSA_RANK_LANES_PER_ROW 1
#endif
constexpr int kRankThreads = BSA_RANK_LANES_PER_ROW * kRankRows;
static_assert(kRankThreads <= 1024, "K2 workgroup size");
__host__ __device__ __forceinline__ int rank_blocks(int nrows) { return (nrows + kRankRows - 1) / kRankRows; }
__host__ __device__ __forceinline__ int rowcnt_words(int nrows) { return 2 * (nrows + 1) + 2 * rank_blocks(nrows); }

// Per-detect state to zero (k_zero, or fused into k_prep_cols: cnt != nullptr)
struct ZeroArgs {
  int nrows, full, keep;
  Counters *cnt;
  unsigned long long *work;
  unsigned char *inconf;
  unsigned long long *tcpamax;
  unsigned *rowcnt;
  unsigned *x[3];  // more word regions to zero (the halo plan's buffers: HaloPre), or NULL
  int xn[3];
};
// Non-finite tcpa inputs (Ctx::nonfin): producers (the column records'
// makers) store `epoch` into *word when a column's position or velocity is
// non-finite; K2 makes every row's tcpamax NaN when *word == epoch, and a
// row's own when rowbad[row] is set (rows of their own, written by
// k_prep_rows in index order; NULL when the rows are columns)
struct NfArgs {
  unsigned long long *word;
  unsigned long long epoch;
  const uint8_t *rowbad;
};

__device__ __forceinline__ bool list_word(int k);
__device__ __forceinline__ void zero_state(const ZeroArgs &z, int t, int nt) {
  constexpr int kWords = (int)(sizeof(Counters) / 8);
  constexpr int kTilesWord = (int)(offsetof(Counters, tiles) / 8);
  constexpr int kNearWord = (int)(offsetof(Counters, tiles_near) / 8);
  const int m = max(max(max(2 * (z.nrows + 1), kWorkShards * kWorkStride), kWords),
                    max(max(z.xn[0], z.xn[1]), z.xn[2]));
  for (int k = t; k < m; k += nt) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
      if (k < z.xn[r]) z.x[r][k] = 0u;
    if (k < kWords && (z.full || (k != kTilesWord && k != kNearWord)) && !(z.keep && list_word(k)))
      reinterpret_cast<unsigned long long *>(z.cnt)[k] = 0;
    if (k < kWorkShards * kWorkStride) z.work[k] = 0;
    if (k < z.nrows) {
      z.inconf[k] = 0;
      z.tcpamax[k] = 0;
    }
    if (k < 2 * (z.nrows + 1)) z.rowcnt[k] = 0;
  }
}


// K0c fused into K0b (no candidate-list reuse): the workgroup's kTile records
// are one tile, so the boxes are reduced right after the records are written.
struct FusedBoxes {
  TileBox *sbox, *gbox, *tbox;  // gbox == nullptr: not fused (k_boxes runs)
  TileBox *blk;                 // halo exchange: tile boxes also into the block sent (blk[tile - blk_base])
  int blk_base;
};

// Plan reuse (several ranks / the probe): the own-tile K0b
// compares each record it writes with the last build's and raises the rank's
// rebuild flag on the first one outside the budgets (snap == NULL: off)
struct TprCheck {
  const PFRec *snap;
  unsigned *flag;
  float dx, ds, dv;
  // HK (Ctx::hk_*): the prediction word of this detect, raised when a record
  // left f x every budget (the list is rebuilt two detects on), or NULL
  unsigned long long *pred;
  float f;
};

// Column records: intruder[j] geometry, own[j] velocity / altitude.
// Workgroup = kTile lanes (one tile of sorted records).  rec = 0 (the
// resident sim's home order): the fp64 records are not stored -- K1b builds
// the few it needs from the state arrays with col_record itself.
// presorted: the state arrays are already in sorted (home) order, perm only
// names the aircraft (the resident sim): record k reads index k, coalesced.
// Tiles: workgroup b prepares tile tile_base + b, or tile_list[b] (a halo
// tile list of the row-sharded step, -1 = unused slot).
// (the waves-per-EU floors below keep the occupancy these kernels had before
// the library's max-ilp scheduling, Makefile: it would trade it for ILP)
__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(6))) void k_prep_cols(int cnt, const unsigned *__restrict__ perm, int presorted, int rec,
                                                     SoA6 own, SoA6 intr, int distinct, int shared,
                                                     double rpz, double hpz, double tla,
                                                     ColRec *__restrict__ C, PFRec *__restrict__ PC,
                                                     PFVel *__restrict__ PV, float4 *__restrict__ PP, int mid,
                                                     ReuseParams rz, FusedBoxes fb, ZeroArgs zs, int tile_base,
                                                     const int *__restrict__ tile_list, HaloUnpack hu,
                                                     Counters *__restrict__ hcnt, TprCheck tck, NfArgs nf, int nown) {
  __shared__ TileBox fgb[kTile / 64];
  // K0z (fused): nothing here reads that state
  if (zs.cnt) zero_state(zs, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
  // workgroups [0, nown): tiles tile_base + b; the rest: slots b - nown of
  // tile_list (the halo K0b's received tiles; one launch with the own tiles
  // when the host kept the plan, HK)
  const int b = (int)blockIdx.x;
  const bool mine = b < nown;
  const int slot = b - nown;
  int tile = mine ? tile_base + b : (hu.count && slot >= (int)*hu.count ? -1 : tile_list[slot]);
  // halo exchange: this slot's received tile rows first (each thread writes
  // the row it prepares below), checked against this rank's plan
  if (!mine && hu.rbuf) tile = halo_unpack_tile(hu, slot, tile, hcnt);
  if (tile < 0) return;  // (the whole workgroup: no barrier is skipped by part of it)
  const int k = tile * kTile + (int)threadIdx.x;
  bool over = false;       // reuse: this aircraft overran a budget
  float use_h = 0.f, use_v = 0.f;
  PFRec pk{}, pb{};        // this lane's record (the fused boxes take it from registers), its build's
  const bool check = tck.snap && mine;  // (the own tiles' records: the halo tiles' are their owners' to check)
  if (check && k < cnt) pb = tck.snap[k];
  if (k < cnt) {
    const int o = presorted ? k : (int)perm[k];
    const double tlap = tla > 0.0 ? tla : 0.0;
    const ColRec c = col_record(own, intr, o);
    if (rec) C[k] = c;
    if (nf.word && !col_tcpa_finite(c)) *nf.word = nf.epoch;
    const double lo = c.lon, sinl = c.sinlat, cosl = c.coslat, gs = own.gs[o], olat = c.olat;
    const double lor = lo * kD2R;
    // (own.lat[j] == 0) leaves the different-hemisphere radius unbounded below
    // when own != intruder (geo.py:128): never prune such a column horizontally
    // nor refine it.
    const bool quirk = distinct && olat == 0.0;
    double coslo, sinlo;
    sincos(lor, &sinlo, &coslo);
    const double px = cosl * coslo, py = cosl * sinlo, pz = sinl;
    float sv = 0.f, sadd = 0.f;
    if (rz.build) {  // reuse (shared records only): budget check against the last build
      double svn = rz.sv_default;
      if (rz.valid) {
        const Snap b = rz.build[k];
        const double dx = px - b.x, dy = py - b.y, dz = pz - b.z;
        const double dch = sqrt(dx * dx + dy * dy + dz * dz);
        const double rho = fmin(sqrt(px * px + py * py), sqrt(b.x * b.x + b.y * b.y));
        // |dE| + |dN| <= (pi/2) |dr| (1 + 2 / rho): the refine basis turns with the row
        const double L = 1.0 + 1.5708 * kRefineChord * (1.0 + 2.0 / rho);
        const double du = c.u - b.u, dv = c.v - b.v;
        const double dh = (dch * 6378137.0 * L + sqrt(du * du + dv * dv) * tlap) * 1.001 + 1e-3;
        const double dvv = (fabs(c.alt - b.alt) + fabs(c.vs - b.vs) * tlap) * 1.001 + 1e-3;
        over = !(dh <= rz.sh) || !(dvv <= (double)b.sv);  // (NaN -> rebuild)
        use_h = (float)fmin(dh / rz.sh, 1e30);
        use_v = (float)fmin(dvv / (double)b.sv, 1e30);
        if (!(use_h >= 0.f)) use_h = 1e30f;
        if (!(use_v >= 0.f)) use_v = 1e30f;
        // next budget: this aircraft's vertical drift rate over ktarget detects
        const double age = (double)rz.ctl[1] + 1.0;
        svn = fmin(rz.sv_max, fmax(rz.sv_min, 2.0 * (dvv / age) * rz.ktarget));
      }
      sv = (float)svn;
      Snap sn;
      sn.x = px;
      sn.y = py;
      sn.z = pz;
      sn.u = c.u;
      sn.v = c.v;
      sn.alt = c.alt;
      sn.vs = c.vs;
      sn.sv = sv;
      sn.pad = 0.f;
      rz.cur[k] = sn;
      sadd = rz.sh_chord;
    }
    // (midpoint mode is never combined with reuse: the host passes mid = 0 then)
    PFRec p = mid ? make_pf_mid(px, py, pz, sinl, cosl, coslo, sinlo, c.u, c.v, gs, c.alt, c.vs, rpz, hpz, tlap)
                  : make_pf(px, py, pz, reach_h(rpz, gs, tlap) + sadd, c.alt,
                            reach_v(hpz, c.vs, c.alt, tlap) + (double)sv, sv);
    if (quirk) p.s = INFINITY;
    PP[k] = make_float4((float)px, (float)py, (float)pz, 0.f);
    PFVel v;
    v.u = (float)c.u;
    v.v = (float)c.v;
    v.vs = (float)c.vs;
    v.flags = (quirk || !(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) ? 1u : 0u;
    // shared records also serve as rows: add the rows' pole flag (k_prep_rows)
    if (shared && !(cosl > 1e-2)) v.flags = 1u;
    PC[k] = p;
    PV[k] = v;
    pk = p;
  }
  if (rz.build) {  // one store per wave, no atomics
    const unsigned long long ob = __ballot(over);
    for (int o = 32; o > 0; o >>= 1) {
      use_h = fmaxf(use_h, __shfl_xor(use_h, o));
      use_v = fmaxf(use_v, __shfl_xor(use_v, o));
    }
    if ((threadIdx.x & 63) == 0) {
      if (ob) rz.ctl[0] = 1u;
      const int wv = k >> 6;
      rz.use[2 * wv] = use_h;
      rz.use[2 * wv + 1] = use_v;
    }
  }
  if (check) {  // plan reuse: one flag store per wave whose records left their budgets
    const bool out = k < cnt && !pf_within(pk, pb, tck.dx, tck.ds, tck.dv);
    if (__ballot(out) && (threadIdx.x & 63) == 0) *tck.flag = 1u;
    if (tck.pred) {  // HK: ... or f x the budgets (a rebuild two detects on)
      const bool near = k < cnt && !pf_within(pk, pb, tck.f * tck.dx, tck.f * tck.ds, tck.f * tck.dv);
      if (__ballot(near) && (threadIdx.x & 63) == 0) *tck.pred = 1ull;
    }
  }
  // K0c (fused): this thread wrote PC[k] above, every thread reaches the barrier
  if (fb.gbox) tile_boxes_v(cnt, tile, pk, fgb, fb.sbox, fb.gbox, fb.tbox);
  if (fb.blk && threadIdx.x == 0) fb.blk[tile - fb.blk_base] = fb.tbox[tile];  // (written by this thread)
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

// Counters words that belong to the candidate list (kept across detects by reuse)
__device__ __forceinline__ bool list_word(int k) {
  constexpr int kCand = (int)(offsetof(Counters, cand) / 8), kTiles = (int)(offsetof(Counters, tiles) / 8);
  constexpr int kGroups = (int)(offsetof(Counters, groups) / 8), kStamp = (int)(offsetof(Counters, stamp) / 8);
  constexpr int kNear = (int)(offsetof(Counters, tiles_near) / 8);
  return k == kCand || k == kTiles || k == kNear || k == kGroups || k >= kStamp;
}

__global__ __launch_bounds__(kTile) __attribute__((amdgpu_waves_per_eu(8))) void k_boxes(int cnt, const PFRec *__restrict__ P,
                                                 TileBox *__restrict__ sbox, TileBox *__restrict__ gbox,
                                                 TileBox *__restrict__ tbox, const unsigned *__restrict__ build,
                                                 Counters *__restrict__ reset) {
  __shared__ TileBox gb[kGroupsPerTile];
  if (build && !build[0]) return;  // reused candidate list: no sweep this detect
  if (reset && blockIdx.x == 0) {  // reuse build: start from an empty candidate list
    constexpr int kWords = (int)(sizeof(Counters) / 8);
    for (int k = threadIdx.x; k < kWords; k += blockDim.x)
      if (list_word(k)) reinterpret_cast<unsigned long long *>(reset)[k] = 0;
  }
  tile_boxes(cnt, blockIdx.x, P, gb, sbox, gbox, tbox);
}

// inclusive wave64 prefix sum on the DPP crossbar (no LDS round trips):
// row_shr 1/2/4/8 within each 16-lane row, then row_bcast 15 / 31 across rows
__device__ __forceinline__ unsigned wave_incl_scan(unsigned x) {
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

// ------------------------------------------------------------------ K0d tile pairs

// K0d: the kept tile pairs, listed in two classes: pairs whose boxes overlap
// ("near": a row tile against itself and its neighbours, the costly items)
// from the front of the list, the others from its back (cap - 1 - k), so the
// sweep dequeues the near pairs first -- longest items first keeps the tail of
// the dynamic schedule short (measured -5 us at box100k).
// Two-level: a workgroup takes one SUPER row (kSuper row tiles), tests its
// union box against every super column's (kSuper column tiles) and only
// expands the kept super pairs into tile pairs: at 1M aircraft ~1 % of the
// (N/512)^2 tile pairs survive, so testing them all (3.8 M box pairs) cost
// 42 us.  A union box is a superset of its tiles' boxes and
// boxes_may_interact is monotone in the extents, so no kept tile pair is
// lost.  One returning atomic per class and expansion round of the
// workgroup (a returning atomic on one word saturates at ~88 per us,
// MI355X_MICROARCH 'dequeue').
constexpr int kTPThreads = 1024;
constexpr int kSuper = 8;  // tiles per super tile (each side)
constexpr int kSlicesPerTile = kTile / kGroup;  // 64-row slices (work items) per row tile
static_assert(kSlicesPerTile == 8, "8 slices per tile (item bit layout, slice boxes = group boxes)");
// present (halo mode, nullable): column tiles whose data this rank holds --
// its own [p0, p1) and the halo tiles it received.  A kept pair with any
// other column tile means the halo plan disagreed with this test (it cannot:
// the plan runs the same boxes_may_interact on the same boxes): it is flagged
// (cnt->halo_miss, the step fails loudly), never silently dropped or swept.
// K0d's test of one (row tile rt, column tile ct) pair: its class (near: the
// boxes overlap, far: they only may interact) and the mask of the row tile's
// 64-row slices whose boxes may reach the column tile (sg: the slice boxes)
__device__ __forceinline__ unsigned tp_classify(const TileBox &a, const TileBox *sg, const TileBox &b, int rt, int ct,
                                                int nrows, int noprune, const uint8_t *__restrict__ present, int p0,
                                                int p1, Counters *__restrict__ cnt, bool &kn, bool &kf) {
  unsigned sm = 0;
  if ((noprune || boxes_may_interact(a, b)) && present && !(ct >= p0 && ct < p1) && !present[ct]) {
    cnt->halo_miss = 1;
  } else if (noprune || boxes_may_interact(a, b)) {
    const bool near = gap(a.lo[0], a.hi[0], b.lo[0], b.hi[0]) == 0.f &&
                      gap(a.lo[1], a.hi[1], b.lo[1], b.hi[1]) == 0.f &&
                      gap(a.lo[2], a.hi[2], b.lo[2], b.hi[2]) == 0.f;
    kn = near;
    kf = !near;
    for (int q = 0; q < kSlicesPerTile; ++q)
      if (rt * kTile + q * kGroup < nrows && (noprune || boxes_may_interact(sg[q], b))) sm |= 1u << q;
  }
  return sm;
}

// K0d's list append of one round (every lane of the NT-lane workgroup calls
// it): the items (slices) of each class and the tile pairs themselves, one
// returning atomic per class (near ones from the front of the list, the
// others from its back)
template <int NT>
__device__ __forceinline__ void tp_emit(bool kn, bool kf, unsigned sm, int rt, int ct, uint2 *__restrict__ out,
                                        unsigned long long cap, Counters *__restrict__ cnt,
                                        unsigned long long *__restrict__ icnt, unsigned (*wpre)[NT / 64],
                                        unsigned long long *bbase) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned ni = (unsigned)__popc(sm);
  const unsigned xn = wave_incl_scan(kn ? ni : 0u), xf = wave_incl_scan(kf ? ni : 0u);
  const unsigned tw = (unsigned)__popcll(__ballot(kn)) | (unsigned)__popcll(__ballot(kf)) << 16;
  if (lane == 63) {
    wpre[0][w] = xn;
    wpre[1][w] = xf;
    wpre[3][w] = tw;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    unsigned run = 0, tiles = 0;
    for (int q = 0; q < NT / 64; ++q) {
      const unsigned v = wpre[threadIdx.x][q];
      wpre[threadIdx.x][q] = run;
      run += v;
      tiles += (wpre[3][q] >> (16 * threadIdx.x)) & 0xffffu;
    }
    bbase[threadIdx.x] = run ? atomicAdd(&icnt[1 + threadIdx.x], (unsigned long long)run) : 0ull;
    if (tiles) {
      atomicAdd(&cnt->tiles, (unsigned long long)tiles);
      if (threadIdx.x == 0) atomicAdd(&cnt->tiles_near, (unsigned long long)tiles);
    }
  }
  __syncthreads();
  if (ni) {  // item = (row tile | slice << 22, column tile); near ones from the front
    unsigned long long k = (kn ? bbase[0] + wpre[0][w] + xn : bbase[1] + wpre[1][w] + xf) - ni;
    for (unsigned m = sm; m; m &= m - 1u, ++k) {
      const uint2 v = make_uint2((unsigned)rt | (unsigned)__builtin_ctz(m) << 22, (unsigned)ct);
      out[kn ? k : cap - 1 - k] = v;
    }
  }
}

__global__ __launch_bounds__(kTPThreads) void k_tilepairs(int nrt, int nct, int nrows, const TileBox *__restrict__ rb,
                                                          const TileBox *__restrict__ rg,
                                                          const TileBox *__restrict__ cb, int noprune,
                                                          uint2 *__restrict__ out, unsigned long long cap,
                                                          Counters *__restrict__ cnt,
                                                          unsigned long long *__restrict__ icnt,
                                                          const unsigned *__restrict__ build,
                                                          const uint8_t *__restrict__ present, int p0, int p1) {
  if (build && !build[0]) return;
  __shared__ TileBox srt[kSuper];                    // this super row's tile boxes
  __shared__ TileBox sgb[kSuper * kSlicesPerTile];   // ... and its 64-row slices' boxes
  __shared__ unsigned keep[kTPThreads];      // kept super columns of the chunk
  __shared__ unsigned wpre[4][kTPThreads / 64];
  __shared__ unsigned long long bbase[2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rt0 = blockIdx.x * kSuper, nr = min(kSuper, nrt - rt0);
  if (threadIdx.x < nr) srt[threadIdx.x] = rb[rt0 + threadIdx.x];
  if (threadIdx.x < nr * kSlicesPerTile && rt0 * kTile + (int)threadIdx.x * kGroup < nrows)
    sgb[threadIdx.x] = rg[rt0 * kSlicesPerTile + threadIdx.x];
  __syncthreads();
  TileBox sr = srt[0];
  for (int i = 1; i < nr; ++i) sr = box_union(sr, srt[i]);
  const int nsc = (nct + kSuper - 1) / kSuper;
  for (int c0 = 0; c0 < nsc; c0 += kTPThreads) {
    // super columns c0 + threadIdx.x: union box, tested against the super row
    const int sc = c0 + threadIdx.x;
    bool kp = false;
    if (sc < nsc) {
      const int ct0 = sc * kSuper, nc = min(kSuper, nct - ct0);
      TileBox u = cb[ct0];
      for (int j = 1; j < nc; ++j) u = box_union(u, cb[ct0 + j]);
      kp = noprune || boxes_may_interact(sr, u);
    }
    const unsigned x = wave_incl_scan(kp ? 1u : 0u);
    if (lane == 63) wpre[2][w] = x;
    __syncthreads();
    unsigned before = 0, K = 0;
    for (int q = 0; q < kTPThreads / 64; ++q) {
      before += q < w ? wpre[2][q] : 0u;
      K += wpre[2][q];
    }
    if (kp) keep[before + x - 1] = (unsigned)sc;
    __syncthreads();
    // expansion: K super columns x (nr row tiles x kSuper column tiles)
    const unsigned ne = K * kSuper * kSuper;
    for (unsigned e0 = 0; e0 < ne; e0 += kTPThreads) {
      const unsigned e = e0 + threadIdx.x;
      bool kn = false, kf = false;
      int rt = 0, ct = 0;
      unsigned sm = 0;  // slices of row tile rt whose boxes may interact with column tile ct
      if (e < ne) {
        const unsigned sc2 = keep[e / (kSuper * kSuper)], r = e % (kSuper * kSuper);
        const int i = (int)(r / kSuper);
        rt = rt0 + i;
        ct = (int)sc2 * kSuper + (int)(r % kSuper);
        if (i < nr && ct < nct) sm = tp_classify(srt[i], &sgb[i * kSlicesPerTile], cb[ct], rt, ct, nrows, noprune,
                                                 present, p0, p1, cnt, kn, kf);
      }
      tp_emit<kTPThreads>(kn, kf, sm, rt, ct, out, cap, cnt, icnt, wpre, bbase);
      __syncthreads();  // wpre / bbase are rewritten by the next round
    }
  }
}

// K0d without the super level, for few column tiles (the 100k box: 196):
// one workgroup per row tile, one lane per column tile -- the super pass's
// union loads, its scan and its barrier were a third of K0d's chain there
constexpr int kTPDirectThreads = 256;
constexpr int kTPDirectMax = 1024;  // column tiles up to which K0d runs direct
// Tile-pair list reuse: ctl == NULL -> off (the list is this
// detect's own); else K0d builds (grown boxes, snapshot of the records) only
// when forced by the host or flagged by the records' preparer (ctl[0]), and
// the prefilter publishes the built list's item counts (ctl[1], ctl[2])
struct TprArgs {
  unsigned long long *ctl;
  int force;
  float dx, ds, dv;
  const PFRec *pc;  // this detect's column records (rows = columns)
  PFRec *snap;
  unsigned *myflag;  // several ranks / the probe: the rank's rebuild flag, cleared here (the plan read it)
  // HK keep (the host kept the list; K0d is not launched): the prefilter takes
  // the kept item counts from ctl[1], ctl[2] and aborts the step
  // (Counters::tpr_stale) when the records' violation word vflag is set
  int keep;
  const unsigned *vflag;
  unsigned long long *stale;  // ... and records it for the batch (sim_ctl, kSimCtlStale)
};

// Halo mode (hl != NULL): the columns are this rank's own tiles [p0, p1) and
// the received halo tiles hl[0, nhl) (-1: an unused slot; *nhl_dev bounds the
// list when set), not all nct tiles -- one rank of 8 at 1M holds ~300 of the
// 1954 tiles.  Every other tile is still tested against the row tile, without
// an append: a kept pair with a tile the halo plan did not deliver sets
// Counters::halo_miss (the step fails loudly), as the full sweep did.
__global__ __launch_bounds__(kTPDirectThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_tilepairs_direct(
    int nrt, int nct, int nrows, const TileBox *__restrict__ rb, const TileBox *__restrict__ rg,
    const TileBox *__restrict__ cb, int noprune, uint2 *__restrict__ out, unsigned long long cap,
    Counters *__restrict__ cnt, unsigned long long *__restrict__ icnt, const unsigned *__restrict__ build,
    const uint8_t *__restrict__ present, int p0, int p1, const TileBox *__restrict__ gbc,
    const int *__restrict__ hl, int nhl, const unsigned *__restrict__ nhl_dev, TprArgs tp) {
  if (tp.myflag && blockIdx.x == 0 && threadIdx.x == 0) *tp.myflag = 0u;  // (k_halo_plan's blocks all read it)
  if (build && !build[0]) return;
  // tile-pair list reuse: no build this detect -> the kept
  // list's item counts into the dequeue words, nothing else
  const bool grow = tp.ctl != nullptr;
  if (grow && !(tp.force || tp.ctl[0] != 0ull)) {
    if (blockIdx.x == 0 && threadIdx.x < 2) icnt[1 + threadIdx.x] = tp.ctl[1 + threadIdx.x];
    return;
  }
  __shared__ TileBox sgb[kSlicesPerTile];
  __shared__ unsigned wpre[4][kTPDirectThreads / 64];
  __shared__ unsigned long long bbase[2];
  const int rt = blockIdx.x;
  // gbc (the resident step's prepped detect, no K0z launch): the tile boxes
  // from the group boxes, as tile_from_groups would have written them (the
  // rows are the columns then, so the row groups are the column groups)
  auto tile_of = [&](int t) {
    const int ng = (nrows + kGroup - 1) / kGroup;  // (all rows detected: nrows = n)
    TileBox g[kGroupsPerTile];
#pragma unroll
    for (int q = 0; q < kGroupsPerTile; ++q) g[q] = gbc[min(t * kGroupsPerTile + q, ng - 1)];  // loads together
    TileBox u = t * kGroupsPerTile < ng ? g[0] : empty_box();
#pragma unroll
    for (int q = 1; q < kGroupsPerTile; ++q) u = box_union(u, t * kGroupsPerTile + q < ng ? g[q] : empty_box());
    return u;
  };
  // column k of the sweep: tile k (all tiles), or own tile p0 + k / halo tile hl[k - (p1 - p0)]
  const int nown = p1 - p0;
  const int ncols = hl ? nown + (nhl_dev ? min(nhl, (int)*nhl_dev) : nhl) : nct;
  auto col_of = [&](int k) { return k >= ncols ? -1 : (!hl ? k : (k < nown ? p0 + k : hl[k - nown])); };
  // every box load issued before the first barrier (one round trip)
  int ct = col_of((int)threadIdx.x);
  TileBox bc = gbc ? tile_of(max(ct, 0)) : cb[max(ct, 0)];
  if (threadIdx.x < kSlicesPerTile && rt * kTile + (int)threadIdx.x * kGroup < nrows)
    sgb[threadIdx.x] = rg[rt * kSlicesPerTile + threadIdx.x];
  TileBox a = gbc ? empty_box() : rb[rt];
  if (grow) {  // a build: the snapshot of this row tile's records (rows = columns here)
    for (int k = rt * kTile + (int)threadIdx.x; k < min(nrows, (rt + 1) * kTile); k += kTPDirectThreads)
      tp.snap[k] = tp.pc[k];
  }
  __syncthreads();
  if (gbc) {  // the row tile's groups are its slices (rows = columns): tile_from_groups' union from LDS
    a = sgb[0];
    for (int q = 1; q < kSlicesPerTile; ++q) a = box_union(a, rt * kTile + q * kGroup < nrows ? sgb[q] : empty_box());
  }
  if (grow) {  // the list outlives this detect: every box grown by the drift budgets
    a = box_grow(a, tp.dx, tp.ds, tp.dv);
    bc = box_grow(bc, tp.dx, tp.ds, tp.dv);
    __syncthreads();  // (every lane has read sgb above)
    if (threadIdx.x < kSlicesPerTile) sgb[threadIdx.x] = box_grow(sgb[threadIdx.x], tp.dx, tp.ds, tp.dv);
    __syncthreads();
  }
  for (int c0 = 0; c0 < ncols; c0 += kTPDirectThreads) {
    if (c0 > 0) {
      ct = col_of(c0 + (int)threadIdx.x);
      if (ct >= 0) bc = gbc ? tile_of(ct) : cb[ct];
      if (grow) bc = box_grow(bc, tp.dx, tp.ds, tp.dv);
    }
    bool kn = false, kf = false;
    unsigned sm = 0;
    if (ct >= 0) sm = tp_classify(a, sgb, bc, rt, ct, nrows, noprune, present, p0, p1, cnt, kn, kf);
    tp_emit<kTPDirectThreads>(kn, kf, sm, rt, ct, out, cap, cnt, icnt, wpre, bbase);
    __syncthreads();  // wpre / bbase are rewritten by the next round
  }
  if (hl) {  // the tiles this rank does not hold: none may be reachable (no appends, no barriers;
             // 4 tiles' loads per lane issued together, not one dependent round trip per tile)
    bool miss = false;
    for (int t0 = (int)threadIdx.x; t0 < nct; t0 += 4 * kTPDirectThreads) {
      TileBox b[4];
      uint8_t pr[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = min(t0 + u * kTPDirectThreads, nct - 1);
        b[u] = cb[t];
        pr[u] = present[t];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int t = t0 + u * kTPDirectThreads;
        miss |= t < nct && !(t >= p0 && t < p1) && !pr[u] && (noprune || boxes_may_interact(a, b[u]));
      }
    }
    if (miss) cnt->halo_miss = 1;
  }
}

__device__ __forceinline__ unsigned long long wave_bcast_u64(unsigned long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ unsigned lane_prefix(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// ------------------------------------------------------------------ K1b pair math (also fused into K1a)
struct PairResult {
  bool conf, los;
  double qdr, dist, tcpa, tin, dcpa;
};

// One (i, j) entry of StateBasedCD.detect + geo.qdrdist_matrix, i != j.
// KWIK (opt-in variant, BSA_FLAG_KWIK): geo.kwikqdrdist_matrix (geo.py:347-363)
// replaces qdrdist_matrix, its metre distance handed over in nm (/ nm) so that
// StateBasedCD.py:22's `* nm` restores metres -- the reference's own detect
// with the geo function swapped (tools/make_golden.py captures exactly that).
template <bool KWIK, bool SC = true>
__device__ __forceinline__ PairResult eval_pair(const RowRec &r, const ColRec &c, double rpz,
                                                double hpz, double tla) {
  PairResult o;
  double qdr, dist_nm;
  if (KWIK) {
    // geo.kwikqdrdist_matrix [i, j]: cavelat at lata[j] + latb[i] (geo.py:355)
    double dist_m;
    kwik_entry(r.lat, r.lon, c.lat, c.lon, c.olat + r.ilat, qdr, dist_m);
    dist_nm = dist_m / kNM;
  } else {
    // geo.qdrdist_matrix (geo.py:118-160)
    qdrdist_entry<SC>(r.lat, r.lon, r.sinlat, r.coslat, r.hemA, c.lat, c.lon, c.sinlat, c.coslat, c.hemA,
                  c.eps, qdr, dist_nm);
  }

  // ---- StateBasedCD.detect (StateBasedCD.py:22-83), off-diagonal entry
  const double dist = dist_nm * kNM + 0.0;
  const double qdrrad = qdr * kD2R;
  double sq, cq;
  sin_cos<SC>(qdrrad, &sq, &cq);
  const double dx = dist * sq;
  const double dy = dist * cq;
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

constexpr int kPayStride = 6;  // doubles per candidate record (cpay): key, qdr, dist, tcpa, tin, dcpa

// The outputs of one evaluated candidate with row buckets (B > 0; K1b and the
// fused pass below): a conflict's 48-B record (word 0 = the column's sorted
// position, so K2's fused MVP reads the intruder's state without an id2h
// lookup) and the pair's (column, candidate) entry in its row's conflict /
// LoS bucket, at the slot the row count's atomic returns (a full bucket raises
// k2_demand: the detect is retried with wider buckets)
__device__ __forceinline__ void exact_bucket(const PairResult &o, int row, unsigned oj, unsigned py,
                                             unsigned long long id, int nrows, int B, double *__restrict__ cpay,
                                             unsigned *__restrict__ rowcnt, uint2 *__restrict__ kb,
                                             Counters *__restrict__ cnt) {
  if (o.conf) {
    double *rec = cpay + id * kPayStride;
    rec[0] = __longlong_as_double((long long)py);
    rec[1] = o.qdr;
    rec[2] = o.dist;
    rec[3] = o.tcpa;
    rec[4] = o.tin;
    rec[5] = o.dcpa;
    const unsigned s = atomicAdd(&rowcnt[row], 1u);
    if (s < (unsigned)B) kb[(size_t)row * B + s] = make_uint2(oj, (unsigned)id);
    else atomicMax(&cnt->k2_demand, (unsigned long long)s + 1);
  }
  if (o.los) {
    const unsigned s = atomicAdd(&rowcnt[nrows + 1 + row], 1u);
    if (s < (unsigned)B) kb[((size_t)nrows + row) * B + s] = make_uint2(oj, (unsigned)id);
    else atomicMax(&cnt->k2_demand, (unsigned long long)s + 1);
  }
}

// K1b fused into the prefilter (stored fp64 records, row
// buckets, not KWIK / candidate reuse): each prefilter workgroup evaluates the
// candidates it appended at the end of its sweep (they sit in its LDS stages),
// and the blocks its waves flushed mid-sweep (a full stage; recorded in LDS).
// A candidate's id (its cpay record, its
// bucket entries) is its slot in the candidate array, shard * ccap + position,
// not K1b's flat index -- K2 reads only what the buckets name.  The candidate
// list, every record and every bucket come out exactly as with K1b's launch
// (the list's order differs, which nothing downstream depends on: K2 ranks
// each row's bucket by column).  R == NULL: K1b runs as its own launch.
struct ExactFuse {
  const RowRec *R;                 // row records (the column records + roff when shared)
  const ColRec *C;                 // column records (sorted / home order)
  const unsigned *perm_r, *perm_c;  // sorted position -> index (perm_r NULL: home rows rb + x)
  double rpz, hpz, tla;
  int rb, nrows, B;
  double *cpay;
  unsigned *rowcnt;
  uint2 *kb;
  unsigned nrec;                   // flush records per wave (<= kFuseRecs; bsa_set_exact_fusion)
};

// One candidate p = (row, sorted column) at slot id: K1b's work for it.
__device__ __forceinline__ void fuse_exact_one(const ExactFuse &xf, uint2 p, unsigned long long id,
                                               Counters *__restrict__ cnt) {
  const unsigned oi = xf.perm_r ? xf.perm_r[p.x] : (unsigned)xf.rb + p.x, oj = xf.perm_c[p.y];
  if (xf.perm_r ? oi == oj : oi == p.y) return;  // an aircraft against itself (never a pair)
  const PairResult o = eval_pair<false, false>(xf.R[p.x], xf.C[p.y], xf.rpz, xf.hpz, xf.tla);  // (sin_cos)
  exact_bucket(o, (int)oi - xf.rb, oj, p.y, id, xf.nrows, xf.B, xf.cpay, xf.rowcnt, xf.kb, cnt);
}


// ------------------------------------------------------------------ K1a prefilter
constexpr int PF_BLOCK = 256;
constexpr int PF_WAVES = PF_BLOCK / 64;

struct RefineParams {
  float R;      // rpz [m]
  float H;      // hpz [m]
  float T;      // max(tla, 0) [s]
  float lim2;   // ((R + EABS) / (1 - E1) / R_S)^2 (unit-sphere units, as the refine's positions)
  float zero;   // 0 (diagnostic builds: -DBSA_PF_REFINE_X2 evaluates the refine twice)
};
constexpr float kRS = 6371000.f;   // scale of the unit-sphere chord to metres
constexpr float kE1 = 0.012f;      // bound on |log(reference dist / estimated dist)|
constexpr float kEABS = 50.f;      // absolute position error budget [m]
// Stage 1 rounding budget (planar test).  Rows lie within
// ~0.02 of the plane origin and a kept pair has s < 0.5, so every term of
// acc is < 0.6 in magnitude and its fp32 roundings (k, K, 1 add, 2 fma; the
// projection errors are inside s's 1e-6 chord margin) total < 2e-7.
constexpr float kPlaneMargin = 4e-7f;

typedef float f2 __attribute__((ext_vector_type(2)));

// stage 2: conservative closest-approach refine of one (row, column) pair.
// rp = (x, y, z, -) and rv = (u, v, vs, alt) of the row, rb = (x, y, rho, -)
// / rho of its fp32 unit vector (its local east / north basis, staged once per
// item); cp = (x, y, z, -) and cv = (u, v, vs, alt) of the column.  Positions
// are unit-sphere chords, u / v are pre-scaled by 1 / R_S (kInvRS) to the
// same units (times and the vertical terms are unchanged).  u is NaN for an
// index that must never be refined (quirk column, non-finite position, row
// within ~0.6 deg of a pole), which keeps the pair through the `vv` test.
// Returns false only when no t in [0, max(tla,0)] can lie in both the
// vertical and the horizontal window of the reference's geometry (DESIGN.md
// "CPA refine"); any NaN keeps the pair.
constexpr float kInvRS = 1.f / kRS;
// far: keep without refining when the chord may exceed kRefineChord.  With
// fp32 unit vectors (|c|^2, |r|^2 within 2e-7 of 1) and the dot product's
// rounding (< 2e-7), chord^2 = |c|^2 + |r|^2 - 2 c.r <= 2 - 2 c.r + 1e-6, so
// c.r >= 1 - (kRefineChord^2 - 2e-6) / 2 refines chords <= kRefineChord only.
constexpr float kFarCos = (float)(1.0 - (kRefineChord * kRefineChord - 2e-6) / 2.0);
__device__ __forceinline__ bool pf_refine(const float4 &rp, const float4 &rv, const float4 &rb, const float4 &cp,
                                          const float4 &cv, const RefineParams &prm) {
  // Branch-free: every lane evaluates every test and the decision is one
  // select at the end -- the same values and the same keep / reject outcome as
  // testing them in order with early returns (far or clamped pairs are kept
  // whatever the rest says), without the exec-mask bookkeeping and the
  // per-branch LDS waits of the early-exit form.
  const bool far = cp.x * rp.x + cp.y * rp.y + cp.z * rp.z < kFarCos;  // > ~190 km: keep
  // the chord projected on the row's local east / north basis
  //   e = (-y, x, 0) / rho,  n = (-z x / rho, -z y / rho, rho),  rho = cos(lat):
  // e.r = n.r = 0, so (c - r).e = c.e and (c - r).n = c.n -- no difference
  // vector, and the per-row basis comes from LDS (|c.e|, |c.n| rounding < 5e-7,
  // ~3 m, inside kEABS)
  const float pe = cp.y * rb.x - cp.x * rb.y;
  const float pn = cp.z * rb.z - rp.z * (cp.x * rb.x + cp.y * rb.y);
  const float ve = cv.x - rv.x, vn = cv.y - rv.y;          // (own.u[j] - int.u[i]) / R_S
  const float vv = ve * ve + vn * vn;
  const bool clamp = !(vv >= 4e-6f * kInvRS * kInvRS);     // reference may clamp dv2; NaN
  const float dalt = cv.w - rv.w;                          // own.alt[j] - int.alt[i]
  const float H = prm.H + (rp.w + cp.w);                   // + vertical budgets (reuse; else 0)
  const float dvs = cv.z - rv.z;
  const float adv = __builtin_fabsf(dvs);
  // reciprocals by v_rcp_f32 (1 ulp): every division here only places a
  // window edge or the closest-approach time, and the margins below are
  // many orders of magnitude wider than 1 ulp
  const bool level = adv < 1e-3f;
  const bool level_out = __builtin_fabsf(dalt) >= H + 1e-3f * prm.T + 2.f + 1e-5f * __builtin_fabsf(dalt);
  const float inv = __builtin_amdgcn_rcpf(dvs);
  const float ta = (-H - dalt) * inv, tb = (H - dalt) * inv;
  const float lo = fminf(ta, tb), hi = fmaxf(ta, tb);
  const float d = (2.f + 1e-5f * (__builtin_fabsf(dalt) + H)) * __builtin_fabsf(inv) +
                  1e-4f * fmaxf(__builtin_fabsf(lo), __builtin_fabsf(hi));
  const float w0 = fmaxf(lo - d, 0.f), w1 = fminf(hi + d, prm.T);
  const bool vout = level ? level_out : (w0 > w1);
  const float t0 = level ? 0.f : w0, t1 = level ? prm.T : w1;
  const float tl = t0 * (1.f - kE1), th = t1 * (1.f + 2.f * kE1);
  float ts = -(pe * ve + pn * vn) * __builtin_amdgcn_rcpf(vv);
  ts = fminf(fmaxf(ts, tl), th);
  const float qe = pe + ve * ts, qn = pn + vn * ts;
  const bool hout = qe * qe + qn * qn > prm.lim2;
  return far | clamp | !(vout | hout);
}

#ifndef PF_Q1
#define PF_Q1 512  // per-wave stage-1 queue: u16 (row_local << 6 | column slot)
#endif
// Refine survivors are staged in the wave's LDS slot of PF_RES candidates; a
// full slot is flushed to the candidate list (one returning atomic on the
// shard counter per PF_RES candidates), and at the end of the sweep the four
// waves of a workgroup flush what is left with ONE atomic together -- the list
// is dense (no unused slots), so K1b runs every wave with all 64 lanes busy
#ifndef PF_RES
#define PF_RES 128
#endif
constexpr int PF_WROWS = 64;   // rows per wave (one per lane)
// fused K1b: mid-sweep flushes a wave can record for the end of its
// workgroup's sweep (each holds >= 65 candidates: >= 4 160 per wave; more sets
// Counters::fuse_ovf and the detect is retried with K1b's own launch)
constexpr int kFuseRecs = kFuseRecsMax;
constexpr int PF_ITEMS_PER_TILE = kTile / PF_WROWS;  // work items per tile pair
// Work distribution knob of the sweep (BSA_PF_SHARDS overrides it for
// measurements; results never depend on it)
struct PfKnobs {
  int pieces;  // units per item (tile pair, 64-row slice): 1, 2, 4 (or 8, BSA_PF_PIECES)
  int pnear;   // ... per near item (the pair's boxes overlap: the densest items)
  int t0;      // log2 of the listed top tier's pieces per near item's (HeavyArgs; BSA_PF_HEAVY_T0)
  // halo overlap (Ctx::ov_mode): 0 every item; 1 the items of the own column
  // tiles [ca0, ca1); 2 the others (the received tiles), with the dequeue
  // counters at word 8 of each shard's stride
  int ph, ca0, ca1;
};
// Longest items first (a kept tile-pair list): the sweep's
// span is set by its longest items (a dense item's refine runs up to ~60 us;
// one that starts late ends long after the median wave).  Every unit adds its
// duration to its list slot's cost; K1b lists the slots above a threshold for
// the next detect (consecutive detects sweep nearly the same pairs), whose
// prefilter dequeues those items first -- split as near items are -- and skips
// them among the regular units (flag == epoch).  Every slot is swept exactly
// once either way: results never depend on which items are listed.
// Two tiers: list 0 (the longest, cost >= thresh[0]) in twice a near item's
// pieces, list 1 (cost >= thresh[1]) split as near items are.
struct HeavyArgs {
  const unsigned *list[2];  // this detect's listed slots, or list[0] NULL (off)
  const unsigned *count;    // ... their numbers [2]
  unsigned *count_next;     // the next detect's [2], zeroed here (K1b appends)
  const unsigned *flag;     // per slot: == epoch -> listed this detect
  unsigned *cost;           // per slot: s_memrealtime ticks of its units (summed)
  unsigned epoch;
};
struct HeavyNext {
  unsigned *cost;           // read and zeroed
  unsigned *list[2], *count, *flag;
  unsigned epoch;           // the next detect's
  unsigned thresh[2];       // ticks (100 MHz)
  const unsigned long long *work;  // [1] near, [2] far items of this detect's list
  unsigned long long icap;
};
#ifndef BSA_PF_WAVES_PER_EU
#define BSA_PF_WAVES_PER_EU 4
#endif
constexpr int PF_BLOCKS_PER_CU = BSA_PF_WAVES_PER_EU;  // resident workgroups per CU (4 waves each): LDS and VGPR limits
constexpr int kSubsPerTile = kTile / kSub;
static_assert(kSubsPerTile == 64, "one sub-group box per lane");
constexpr int kSubsPerBatch = 64 / kSub;  // sub-groups per 64-column batch
static_assert(PF_Q1 >= 64 * 8, "one 8-column chunk of survivors fits the stage-1 queue");

// Diagnostic item timeline (build with -DBSA_PF_TRACE; `make trace`,
// tools/pf_trace.py): per work item {item, wave << 8 | sub-groups, start,
// end} (s_memrealtime, 100 MHz) into a per-wave region of pf_trace (no
// atomics), dumped by detect_finish to $BSA_PF_TRACE_FILE.
#ifdef BSA_PF_TRACE
__device__ unsigned long long *pf_trace;
constexpr unsigned long long kTraceRecs = 1ull << 21;
constexpr unsigned kTraceWave = 256;
#endif
// Diagnostic phase timers (build with -DBSA_PF_STAMPS; `make stamps`):
// cycles per wave spent in 0 dequeue/setup, 1 stage 1, 2 refine drains,
// 3 flushes, summed over waves into Counters::stamp.
#ifdef BSA_PF_STAMPS
#define PF_STAMP(k)                                               \
  do {                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += now_ - st_last;                                  \
    st_last = now_;                                               \
  } while (0)
#else
#define PF_STAMP(k) \
  do {              \
  } while (0)
#endif

// K1a: each wave sweeps its 64 rows (one per lane, in registers) against the
// columns of a tile pair that survive culling at 8-column sub-group
// granularity (each lane tests one of the 64 sub-group boxes of the
// 512-column tile against the wave's row box).  The surviving columns are
// gathered in batches of 64 (eight sub-groups; one coalesced record load per lane, issued
// one batch ahead), projected and staged in the wave's LDS slot as column
// PAIRS, from which every lane reads them as broadcasts: each packed fp32
// instruction tests the lane's row against two columns.
//
// Stage 1 works in a plane: rows and columns are projected orthogonally onto
// the plane spanned by an (fp32-)orthonormal pair E, N (the tangent plane at
// the item's first row).  A projection never lengthens a vector, so the planar
// distance is <= the chord and "planar < s_i + s_j" keeps every pair with
// chord < s_i + s_j, wherever E, N point.  With P = ((p - o).E, (p - o).N) and
// k = s^2/2 - |P|^2/2 the test is linear in the column's values:
//   acc = (K_i + k_j) + s_i s_j + E_i e_j + N_i n_j = ((s_i + s_j)^2 - |P_i - P_j|^2) / 2
// (K_i = k_i + kPlaneMargin), plus the vertical interval test
// lo_j < hi_i and hi_j > lo_i.  The three signs are combined with one
// v_bitop3 (keep iff sign(acc) = 0, sign(lo_j - hi_i) = 1, sign(hi_j - lo_i) = 0;
// the +-0 and NaN cases can only keep a pair, never drop one) and shifted
// into a per-lane column bit mask with v_alignbit.
//
// Survivors of each 8-column chunk go to an LDS queue (DPP prefix sum of the
// per-lane counts).  The queue is drained after every batch (or when full)
// with all 64 lanes busy through stage 2 (refine) on LDS-resident inputs (the
// batch's staged columns, the item's staged rows, row unit vectors by
// ds_bpermute).  Stage-2 survivors are staged in the wave's LDS slot and
// appended densely to the candidate list (one atomic per PF_RES candidates,
// and one per workgroup at the end of the sweep).
template <bool NOPRUNE>
// 4 waves per SIMD = PF_BLOCKS_PER_CU resident workgroups: up to 128 VGPRs,
// no spills (at 5 waves the 96-VGPR cap spilled to scratch, and every scratch
// reload in the batch loop waited for the in-flight prefetch: 8 us slower)
#define PF_OCC __attribute__((amdgpu_waves_per_eu(BSA_PF_WAVES_PER_EU, 8)))
__global__ __launch_bounds__(PF_BLOCK) PF_OCC void k_prefilter(
    const PFRec *__restrict__ prow, const PFVel *__restrict__ vrow, const float4 *__restrict__ pprow, int nrows,
    const PFRec *__restrict__ pcol, const PFVel *__restrict__ vcol, const float4 *__restrict__ ppcol, int ncols,
    const TileBox *__restrict__ gbox_r, const TileBox *__restrict__ sbox_c, int noprune,
    const uint2 *__restrict__ items, unsigned long long icap,
    Counters *__restrict__ cnt,
    unsigned long long *__restrict__ work, RefineParams prm,
    uint2 *__restrict__ cand, unsigned long long cap, const unsigned *__restrict__ build, PfKnobs kn, int diag,
    TprArgs tp, HeavyArgs hv, ExactFuse xf) {
  __shared__ unsigned short q1s[PF_WAVES][PF_Q1];
  __shared__ float4 cka[PF_WAVES][32];      // staged column pairs: k k' s s'     (stage 1)
  __shared__ float4 cen[PF_WAVES][32];      //                      e e' n n'     (stage 1)
  __shared__ float4 clh[PF_WAVES][32];      //                      lo lo' hi hi' (stage 1)
  __shared__ float4 csx[PF_WAVES][64];      // staged columns:      x y z -       (refine)
  __shared__ float4 csv[PF_WAVES][64];      //                      u v vs alt    (refine)
  __shared__ unsigned cix[PF_WAVES][64];    //                      sorted column index
  __shared__ float4 rsv[PF_WAVES][PF_WROWS];  // staged rows:       u v vs alt    (refine)
  __shared__ float4 rsp[PF_WAVES][PF_WROWS];  //                    x y z sigma   (refine)
  __shared__ float4 rbs[PF_WAVES][PF_WROWS];  //                    x/rho y/rho rho - (refine basis)
  __shared__ unsigned char sgs[PF_WAVES][kSubsPerBatch];  // the next batch's sub-groups (tile-local)
  __shared__ uint2 cst[PF_WAVES][PF_RES];   // staged candidates (row, column) of the wave
  if (build && !build[0]) return;  // reused candidate list
  if (tp.keep && *tp.vflag != 0u) {  // HK: a record left the kept list's budgets -- the step re-runs
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      cnt->tpr_stale = 1ull;
      if (tp.stale) *tp.stale = 1ull;  // (the batch's own record: later detects' counters may not show it)
    }
    // (the next detect's listed-item counts start at zero as in a sweep:
    // this detect's K2 still lists items for it, and a stale count would
    // sweep old slots twice)
    if (hv.list[0] && blockIdx.x == 0 && threadIdx.x < 2) hv.count_next[threadIdx.x] = 0u;
    return;
  }
  if (tp.ctl && kn.ph != 2 && blockIdx.x == 0 && threadIdx.x == 0) {  // tile-pair list reuse: K0d is complete here
    if (!tp.keep && (tp.force || tp.ctl[0] != 0ull)) {  // it built: keep the list's counts, clear the flag
      tp.ctl[1] = work[1];
      tp.ctl[2] = work[2];
      tp.ctl[0] = 0ull;
      tp.ctl[3] += 1ull;
    }
    tp.ctl[4] += 1ull;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  unsigned short *q1 = q1s[w];
  float *ska = (float *)cka[w];
  float *sen = (float *)cen[w];
  float *slh = (float *)clh[w];
  float4 *sx = csx[w];
  float4 *sv = csv[w];
  unsigned *sci = cix[w];
  float4 *rv = rsv[w];
  unsigned subs = 0;      // 8-column sub-groups swept by this wave (for the roofline)
  const float qnan = __builtin_nanf("");
  // Dynamic work distribution: an item is one (tile pair, 64-row slice) that
  // K0d listed (the slice's box may reach the column tile's: at the 100k box
  // 44 % of the 8 x 3 642 slices do not, and each cost its wave a dequeue ->
  // tile -> box-load chain when all were numbered implicitly), split into
  // `pieces` units; each wave dequeues units from the counter of its shard
  // (blockIdx % 32, 128 B apart; a returning atomic on one word saturates at
  // ~88 per us).  Near tile pairs (the costly ones) come first in the list.  A
  // unit's sub-group mask is formed as it starts (below).  (Measured slower:
  // claiming the next item ahead (+20 us, also without spills: a returning
  // atomic in flight joins every later in-order vmcnt wait, so its latency is
  // moved, not hidden); several items per dequeue, or PF_GROUP consecutive tile
  // pairs of one slice per item sharing the row setup, with the next pair's
  // first batch prefetched (+10 / +30 / +90 us at 2 / 4 / 8: fewer, longer
  // items balance worse); stealing items from other shards once a wave's shard
  // is dry (+130 us: the drained shards' counters are hammered by failing
  // returning atomics); a separate K0e launch listing only the items with a
  // non-empty sub-group mask, dense ones split further (-8 us of sweep, but the
  // launch's cold dependent loads took 13 us).)
  // pieces > 1: a unit takes the set bits of rank p mod pieces of its item's
  // column mask (an equal share of the sub-groups; contiguous quarters of the
  // mask were uneven where the dense columns bunch) -- the densest items, 60-85
  // us each, set the sweep's span otherwise (tools/pf_trace.py); empty pieces
  // are skipped
  // K0d's items (complete before this launch): near ones from the front of
  // the list, the others from its back; each is `pieces` units
  // near items take kn.pnear units each, the others kn.pieces
  // (32-bit unit arithmetic, powers of two: the 64-bit forms with a run-time
  // divisor expanded into ~50 scalar instructions per unit)
  const unsigned lnear = (unsigned)__builtin_ctz((unsigned)kn.pnear), lpc = (unsigned)__builtin_ctz((unsigned)kn.pieces);
  // (HK keep: no K0d copied the kept list's counts into the dequeue words)
  const unsigned inear = (unsigned)(tp.keep ? tp.ctl[1] : work[1]), unear = inear << lnear;
  const unsigned nfar = (unsigned)(tp.keep ? tp.ctl[2] : work[2]);
  const unsigned nreg = unear + (nfar << lpc);
  unsigned nh0 = 0, nh1 = 0;
  if (hv.list[0]) {
    nh0 = __builtin_amdgcn_readfirstlane(hv.count[0]);
    nh1 = __builtin_amdgcn_readfirstlane(hv.count[1]);
    if (blockIdx.x == 0 && threadIdx.x < 2) hv.count_next[threadIdx.x] = 0u;
  }
  const unsigned lh0 = lnear + (unsigned)kn.t0;
  const unsigned hu0 = nh0 << lh0, hunits = hu0 + (nh1 << lnear);
  const unsigned nunits = hunits + nreg;
  const unsigned shard = blockIdx.x & (kWorkShards - 1);
  unsigned long long *wq = work + shard * kWorkStride + (kn.ph == 2 ? 8 : 0);
  // candidates: shard `shard` owns cand[shard * ccap, (shard + 1) * ccap) and
  // its own counter (spreads the flush atomics over kCandShards addresses)
  const unsigned long long ccap = cap / kCandShards;
  uint2 *ccand = cand + (unsigned long long)(shard % kCandShards) * ccap;
  unsigned long long *cshard = &cnt->cshard[shard % kCandShards][0];
  // the wave's staged candidates cst[w][0, nst) (wave-uniform count): a refine
  // round's survivors (mask mk) take the next entries in lane order; a round
  // that does not fit flushes the slot first (one returning atomic on the
  // shard counter reserves exactly nst list slots).  Most waves never flush
  // before the end of the sweep (the 100k box: ~37 candidates per wave), where
  // the workgroup flushes its four slots with one atomic.  (Reserving blocks of
  // PF_RES list slots directly left each wave's last block ~70 % unused: K1b
  // ran ~524 k slots for ~153 k candidates.)
  // (32-bit slot arithmetic: a shard's slots, and its counter until an
  // overflowing detect is retried, stay far below 2^32)
  const unsigned ccap32 = (unsigned)ccap;
  uint2 *stg = cst[w];
  unsigned nst = 0;
  unsigned nemit = 0;  // candidates this wave wrote (statistics)
  // fused K1b: the blocks this wave flushed mid-sweep, {position, count} (wave-uniform count)
  __shared__ uint2 xrc[PF_WAVES][kFuseRecs];
  unsigned nxr = 0;
  auto flush_stage = [&]() {
    __builtin_amdgcn_wave_barrier();
    unsigned long long r = 0;
    if (lane == 0) r = atomicAdd(cshard, (unsigned long long)nst);
    const unsigned nb = __builtin_amdgcn_readfirstlane((unsigned)r);
    for (unsigned k = lane; k < nst; k += 64)
      if (nb + k < ccap32) ccand[nb + k] = stg[k];
    if (xf.R) {  // fused K1b: the block is evaluated at the end of the workgroup's sweep
      if (lane == 0) {
        if (nxr < xf.nrec) xrc[w][nxr] = make_uint2(nb, nst);
        else cnt->fuse_ovf = 1ull;  // (the detect is retried with K1b as its own launch)
      }
      ++nxr;
    }
    nst = 0;
    __builtin_amdgcn_wave_barrier();
  };
  auto emit = [&](unsigned long long mk, bool keep, uint2 v) {
    const unsigned c = (unsigned)__popcll(mk), pre = lane_prefix(mk);
    if (nst + c > (unsigned)PF_RES) flush_stage();
    if (keep) stg[nst + pre] = v;
    nst += c;
    nemit += c;
  };
#ifdef BSA_PF_STAMPS
  // [4] stage-1 survivors, [5] refine rounds, [6] batches, [7] enqueue loop trips
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_last = __builtin_amdgcn_s_memtime();
#endif
#ifdef BSA_PF_TRACE
  unsigned tr_n = 0;
#endif
  for (;;) {
    unsigned item;
    {
      unsigned long long m0 = 0;
      if (lane == 0) m0 = atomicAdd(wq, 1ull);
      item = __builtin_amdgcn_readfirstlane((unsigned)m0);
    }
    // the unit of the shard's item-th dequeue: blocks of 8 consecutive units, 4
    // consecutive blocks to the 4 shards of one XCD (shard & 7 = the XCD of its
    // workgroups), so the items of a tile pair -- consecutive in the list -- are
    // swept on one XCD, close together in time: the column tile enters one L2
    item = (((item >> 3) * kWorkShards + 4 * (shard & 7) + (shard >> 3)) << 3) | (item & 7u);
    if (item >= nunits) break;
#ifdef BSA_PF_TRACE
    const unsigned long long tr0 = __builtin_amdgcn_s_memrealtime();
    unsigned tr_subs = 0;
#endif
    // the unit's list slot and piece: a listed item's piece (the first hunits
    // units), or a regular unit -- skipped when its item is listed
    unsigned long long slot;
    unsigned ls, piece;
    bool skip = false;
    const unsigned long long hq0 = hv.cost ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (item < hunits) {
      const bool t0 = item < hu0;
      ls = t0 ? lh0 : lnear;
      const unsigned ui = t0 ? item : item - hu0;
      piece = ui & ((1u << ls) - 1u);
      slot = hv.list[t0 ? 0 : 1][ui >> ls];
      skip = !(slot < inear || (slot >= icap - nfar && slot < icap));  // (a slot of a list since rebuilt)
      if (skip) slot = 0;
    } else {
      const unsigned uj = item - hunits;
      const bool inr = uj < unear;
      ls = inr ? lnear : lpc;
      const unsigned ui = inr ? uj : uj - unear;
      piece = ui & ((1u << ls) - 1u);
      const unsigned e = inr ? (ui >> ls) : inear + (ui >> ls);
      slot = e < inear ? (unsigned long long)e : icap - 1 - (unsigned long long)(e - inear);
      if (hv.list[0]) skip = hv.flag[slot] == hv.epoch;
    }
    const unsigned npc = 1u << ls;
    const uint2 it = items[slot];  // (issued with the flag's load: the skip needs both)
    if (kn.ph && !skip)  // halo overlap: the other launch sweeps it
      skip = ((it.y - (unsigned)kn.ca0) < (unsigned)(kn.ca1 - kn.ca0)) != (kn.ph == 1);
    do {  // one item; `break` ends it
    if (skip) break;
    // the item: (row tile | slice << 22, column tile)
    const uint2 rc = make_uint2(it.x & 0x3fffffu, it.y);
    const unsigned slice = it.x >> 22;
    // column sub-groups of this tile that may interact with the wave's row box:
    // the stage-1 test on box gaps (one sub-group box per lane), evaluated as
    // the item starts
    unsigned long long gm;
    {
      const int cb = (int)rc.y * kTile;
      const int nsub = min(kSubsPerTile, (ncols - cb + kSub - 1) / kSub);
      const int sg = min(lane, nsub - 1);
      const TileBox sb = sbox_c[cb / kSub + sg];
      const TileBox rg = gbox_r[((int)rc.x * kTile) / kGroup + (int)slice];
      gm = __ballot(lane < nsub && (noprune || boxes_may_interact(rg, sb)));
    }
    if (npc > 1)  // piece p: the set bits of rank p, p + npc, ... (equal shares of a dense mask)
      gm = __ballot(((gm >> lane) & 1ull) && (lane_prefix(gm) & (npc - 1u)) == piece);
    const int rbase = (int)rc.x * kTile + (int)slice * PF_WROWS;
    const int cbase = (int)rc.y * kTile;
    if (!gm) break;
    subs += (unsigned)__popcll(gm);
#ifdef BSA_PF_TRACE
    tr_subs = (unsigned)__popcll(gm);
#endif

    // the next batch = the first kSubsPerBatch remaining sub-groups (ascending):
    // lane b holding the r-th set bit of m (r < 8, r = set bits below b) posts
    // b to slot r; this lane takes column lane % kSub of the sub-group in slot
    // lane / kSub.  `taken` = the batch's bits, removed from the mask after it.
    unsigned long long taken = 0;
    auto batch_col = [&](unsigned long long m) -> int {
      const bool mine = ((m >> lane) & 1ull) && lane_prefix(m) < (unsigned)kSubsPerBatch;
      if (mine) sgs[w][lane_prefix(m)] = (unsigned char)lane;
      taken = __ballot(mine);
      const unsigned q = (unsigned)lane / kSub;
      if (q >= (unsigned)__popcll(taken)) return -1;
      const int j = cbase + (int)sgs[w][q] * kSub + (lane & (kSub - 1));
      return j < ncols ? j : -1;
    };
    auto drop_batch = [&](unsigned long long m) { return m & ~taken; };
    // unconditional loads (an empty slot reads column 0; its survivor bits are
    // masked by colmask and it is never queued): a load under a branch makes
    // the compiler wait for it right there, which would expose the prefetch
    auto load_col = [&](int j, PFRec &r, PFVel &v, float4 &q) {
      const int jj = j >= 0 ? j : 0;
      r = pcol[jj];
      v = vcol[jj];
      q = ppcol[jj];
    };
    int jn = batch_col(gm);
    PFRec nx;
    PFVel nv;
    float4 np;
    load_col(jn, nx, nv, np);

    const int krow = rbase + lane;
    const bool va = krow < nrows;
    // (unconditional, as load_col: a lane past the last row reads row rbase and
    // its survivor bits are masked)
    const int krw = va ? krow : rbase;
    const PFRec A = prow[krw];
    const PFVel AV = vrow[krw];
    const float4 AP = pprow[krw];
    // the item's plane: o = first row of the slice, E / N an orthonormal
    // tangent pair at o (any orthonormal pair is exact-safe; near a pole, or
    // for a non-finite o, the x / y axes)
    // (wave-uniform: kept in SGPRs)
    PFRec O = prow[rbase];
    O.x = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(O.x)));
    O.y = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(O.y)));
    O.z = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(O.z)));
    float ex = 1.f, ey = 0.f, nxx = 0.f, nyy = 1.f, nzz = 0.f;
    {
      const float rho2 = O.x * O.x + O.y * O.y;
      if (rho2 > 1e-6f && rho2 <= 1.f) {
        const float ir = __builtin_amdgcn_rsqf(rho2);
        const float rho = rho2 * ir;
        ex = -O.y * ir;
        ey = O.x * ir;
        nxx = -O.z * O.x * ir;
        nyy = -O.z * O.y * ir;
        nzz = rho;
      }
    }
    const float ox = isfinite(O.x) ? O.x : 0.f, oy = isfinite(O.y) ? O.y : 0.f,
                oz = isfinite(O.z) ? O.z : 0.f;
    auto project = [&](float x, float y, float z, float &e, float &n) {
      const float dx = x - ox, dy = y - oy, dz = z - oz;
      e = dx * ex + dy * ey;
      n = dx * nxx + dy * nyy + dz * nzz;
    };
    float re_, rn_;
    project(A.x, A.y, A.z, re_, rn_);
    const f2 E = {re_, re_}, N = {rn_, rn_}, S = {A.s, A.s};
    const float kr = 0.5f * A.s * A.s - 0.5f * (re_ * re_ + rn_ * rn_) + kPlaneMargin;
    const f2 K = {kr, kr};
    const f2 HI = {A.hi, A.hi}, LO = {A.lo, A.lo};
    // the row of this lane for the refine (u = NaN: never refine), position at
    // t = 0 and vertical budget; read from LDS by the drain (a register
    // broadcast would make it wait for the in-flight batch prefetch)
    rv[lane] = make_float4(AV.flags ? qnan : AV.u * kInvRS, AV.v * kInvRS, AV.vs, A.alt);
    rsp[w][lane] = make_float4(AP.x, AP.y, AP.z, A.pad);
    {  // the row's refine basis (rows within ~0.6 deg of a pole are flagged: u = NaN)
      const float rho2 = AP.x * AP.x + AP.y * AP.y;
      const float irho = __builtin_amdgcn_rsqf(rho2);
      rbs[w][lane] = make_float4(AP.x * irho, AP.y * irho, rho2 * irho, 0.f);
    }
    unsigned n1 = 0;                 // wave-uniform
    unsigned long long colmask = 0;  // valid slots of the swept batch

    auto drain = [&]() {
      __builtin_amdgcn_wave_barrier();
      PF_STAMP(1);
#ifdef BSA_PF_STAMPS
      st_acc[4] += n1;
      st_acc[5] += (n1 + 63) / 64;
#endif
      for (unsigned b0 = 0; b0 < n1; b0 += 64) {
        const unsigned k = b0 + lane;
        const unsigned e = q1[k < n1 ? k : b0];
        const unsigned rl = e >> 6, cl = e & 63u;
        bool keep = false;
        unsigned gi = 0, gj = 0;
        if (k < n1) {
          gi = (unsigned)rbase + rl;
          gj = sci[cl];
          keep = NOPRUNE ? true : pf_refine(rsp[w][rl], rv[rl], rbs[w][rl], sx[cl], sv[cl], prm);
          // an aircraft against itself (rows = the columns [diag, diag + nrows)):
          // never a pair (StateBasedCD.py's +1e9 I sentinel), ~40 % of the
          // refine survivors at the 100k box otherwise
          keep = keep && (diag < 0 || gj != (unsigned)diag + gi);
#ifdef BSA_PF_REFINE_X2
          {  // the same test on inputs the compiler cannot prove equal: the refine's cost, measured
            float4 c2 = sx[cl];
            c2.x += prm.zero;
            keep = keep & (NOPRUNE ? true : pf_refine(rsp[w][rl], rv[rl], rbs[w][rl], c2, sv[cl], prm));
          }
#endif
        }
        const unsigned long long mk = __ballot(keep);
        if (mk) {
          emit(mk, keep, make_uint2(gi, gj));
        }
      }
      n1 = 0;
      __builtin_amdgcn_wave_barrier();
      PF_STAMP(2);
    };

    // survivors of 8-column chunk(s) arrive as a per-lane bit mask (bit u =
    // slot col0 + u); `enqueue` queues one chunk (the rare path when a whole
    // batch overflows the queue)
    auto enqueue = [&](unsigned bm, unsigned col0) {
      const unsigned c = (unsigned)__popc(bm);
      const unsigned x = wave_incl_scan(c);
      const unsigned total = __builtin_amdgcn_readlane(x, 63);
      if (total == 0) return;
      if (n1 + total > (unsigned)PF_Q1) drain();
      unsigned pos = n1 + x - c;
#ifdef BSA_PF_STAMPS
      {
        unsigned mx = c;
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
        st_acc[7] += mx;
      }
#endif
      while (bm) {
        q1[pos++] = (unsigned short)(((unsigned)lane << 6) | (col0 + (unsigned)__builtin_ctz(bm)));
        bm &= bm - 1u;
      }
      n1 = __builtin_amdgcn_readfirstlane(n1 + total);
    };
    // the whole batch's survivors (bit = slot) with ONE wave scan; the queue is
    // empty here (drained after every batch)
    auto enqueue_batch = [&](unsigned long long M) {
      const unsigned c = (unsigned)__popcll(M);
      const unsigned x = wave_incl_scan(c);
      const unsigned total = __builtin_amdgcn_readlane(x, 63);
      if (total == 0) return;
      if (total > (unsigned)PF_Q1) {
#pragma unroll 1
        for (unsigned ch = 0; ch < 8; ++ch) enqueue((unsigned)(M >> (8 * ch)) & 0xffu, 8 * ch);
        return;
      }
      unsigned pos = x - c;
      while (M) {
        q1[pos++] = (unsigned short)(((unsigned)lane << 6) | (unsigned)__builtin_ctzll(M));
        M &= M - 1ull;
      }
      n1 = total;
    };

    PF_STAMP(0);
    for (;;) {
      // project and stage the current batch (in-order LDS within the wave:
      // these writes land after the previous batch's reads, incl. its drain)
      {
        float ce, cn;
        project(nx.x, nx.y, nx.z, ce, cn);
        const float ck = 0.5f * nx.s * nx.s - 0.5f * (ce * ce + cn * cn);
        const int pb = (lane >> 1) * 4 + (lane & 1);  // pair lane>>1, half lane&1
        ska[pb] = ck;
        ska[pb + 2] = nx.s;
        sen[pb] = ce;
        sen[pb + 2] = cn;
        slh[pb] = nx.lo;
        slh[pb + 2] = nx.hi;
        sx[lane] = make_float4(np.x, np.y, np.z, nx.pad);
        sv[lane] = make_float4(nv.flags ? qnan : nv.u * kInvRS, nv.v * kInvRS, nv.vs, nx.alt);
        sci[lane] = (unsigned)jn;
        colmask = __ballot(jn >= 0);
      }
#ifdef BSA_PF_STAMPS
      st_acc[6] += 1;
#endif
      gm = drop_batch(gm);
      const bool more = gm != 0;
      // prefetch the next batch while this one is swept (unconditionally: see load_col)
      jn = more ? batch_col(gm) : -1;
      load_col(jn, nx, nv, np);
      // sweep only the chunks holding valid slots
      const int nchunk = colmask ? (64 - __builtin_clzll(colmask) + 7) >> 3 : 0;
      // the survivor bits of chunks 0-3 / 4-7 shift into one word each (four
      // chunks unrolled: static LDS offsets, and the bit reversal / 64-bit
      // placement once per four chunks instead of per chunk)
      unsigned long long M = 0;  // this lane's stage-1 survivors of the batch, bit = slot
#pragma unroll 1
      for (int hf = 0; hf < 2; ++hf) {
      const int kc = min(max(nchunk - 4 * hf, 0), 4);
      if (!kc) break;
      unsigned bm = 0;
#pragma unroll
      for (int c4 = 0; c4 < 4; ++c4) {
        if (c4 >= kc) break;
        const int j0 = (hf * 4 + c4) * 8;
#pragma unroll
        for (int h = 0; h < 4; h += 2) {
        // two column pairs per load group (register pressure: occupancy)
        float4 pa[2], pe[2], pl[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          pa[u] = cka[w][(j0 >> 1) + h + u];
          pe[u] = cen[w][(j0 >> 1) + h + u];
          pl[u] = clh[w][(j0 >> 1) + h + u];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (NOPRUNE) {
            bm = (bm << 2) | 3u;
          } else {
            f2 acc = K + (f2){pa[u].x, pa[u].y};
            acc = __builtin_elementwise_fma(S, (f2){pa[u].z, pa[u].w}, acc);
            acc = __builtin_elementwise_fma(E, (f2){pe[u].x, pe[u].y}, acc);
            acc = __builtin_elementwise_fma(N, (f2){pe[u].z, pe[u].w}, acc);
            const f2 dlo = (f2){pl[u].x, pl[u].y} - HI;   // < 0 to keep
            const f2 dhi = (f2){pl[u].z, pl[u].w} - LO;   // > 0 to keep
            const unsigned t0 = (unsigned)__float_as_int(dlo.x) &
                                ~((unsigned)__float_as_int(acc.x) | (unsigned)__float_as_int(dhi.x));
            const unsigned t1 = (unsigned)__float_as_int(dlo.y) &
                                ~((unsigned)__float_as_int(acc.y) | (unsigned)__float_as_int(dhi.y));
            bm = __builtin_amdgcn_alignbit(bm, t0, 31);   // (bm << 1) | (t0 >> 31)
            bm = __builtin_amdgcn_alignbit(bm, t1, 31);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        }
      }
      // bit 8 kc - 1 - u <-> slot 32 hf + u: reverse into bit u
      M |= (unsigned long long)(__builtin_bitreverse32(bm) >> (32 - 8 * kc)) << (32 * hf);
      }
      enqueue_batch(M & colmask & (va ? ~0ull : 0ull));
      // refine this batch's survivors while its columns are staged
      if (n1) drain();
      PF_STAMP(1);
      if (!more) break;
    }
    } while (0);
    if (hv.cost && lane == 0 && !skip)  // (non-returning)
      atomicAdd(&hv.cost[slot], (unsigned)(__builtin_amdgcn_s_memrealtime() - hq0));
#ifdef BSA_PF_TRACE
    if (lane == 0 && pf_trace) {  // per-wave record region (no atomics)
      const unsigned long long slot = ((unsigned long long)blockIdx.x * PF_WAVES + w) * kTraceWave + tr_n++;
      if (tr_n <= kTraceWave && slot < kTraceRecs) {
        unsigned long long *t = pf_trace + 4 * slot;
        t[0] = item | (item < hunits ? (1ull << 63) : 0ull) | ((unsigned long long)npc << 48);  // listed, pieces
        t[1] = ((unsigned long long)blockIdx.x << 2 | w) << 8 | tr_subs;
        t[2] = tr0;
        t[3] = __builtin_amdgcn_s_memrealtime();
      }
    }
#endif
  }
  PF_STAMP(0);
  // the workgroup's staged candidates with one atomic on its shard counter,
  // and the roofline's sub-group count: one atomic per workgroup, spread over
  // 32 lines (4096 waves adding to one word serialised at ~12 ns each, ~50 us
  // of the sweep's tail when the waves finish together)
  __shared__ unsigned wsubs[PF_WAVES], wcand[PF_WAVES], wst[PF_WAVES], wxr[PF_WAVES];
  __shared__ unsigned wbase;
  if (lane == 0) {
    wsubs[w] = subs;
    wcand[w] = nemit;
    wst[w] = nst;
    wxr[w] = min(nxr, xf.nrec);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned t = 0, tc = 0, ts = 0;
    for (int q = 0; q < PF_WAVES; ++q) t += wsubs[q];
    if (t) atomicAdd(&cnt->gpart[blockIdx.x & 31][0], (unsigned long long)t);
    for (int q = 0; q < PF_WAVES; ++q) tc += wcand[q];
    if (tc) atomicAdd(&cnt->gpart[blockIdx.x & 31][1], (unsigned long long)tc);  // candidates
    for (int q = 0; q < PF_WAVES; ++q) ts += wst[q];
    wbase = ts ? (unsigned)atomicAdd(cshard, (unsigned long long)ts) : 0u;
  }
  __syncthreads();
  if (!xf.R) {  // (fused K1b: nothing reads the final candidates back from the list)
    unsigned o = wbase;
    for (int q = 0; q < w; ++q) o += wst[q];
    for (unsigned k = lane; k < nst; k += 64)
      if (o + k < ccap32) ccand[o + k] = stg[k];
  } else {  // fused K1b (ExactFuse)
    // the workgroup's own final candidates [wbase, wbase + ts) of its shard,
    // from its waves' LDS stages (all 256 lanes: ~150 candidates at the 100k box)
    const unsigned o1 = wst[0], o2 = o1 + wst[1], o3 = o2 + wst[2], ts = o3 + wst[3];
    const unsigned long long sbase = (unsigned long long)(shard % kCandShards) * ccap;
    for (unsigned k = threadIdx.x; k < ts; k += PF_BLOCK) {
      const int q = (k >= o1) + (k >= o2) + (k >= o3);
      const unsigned kq = k - (q == 0 ? 0u : (q == 1 ? o1 : (q == 2 ? o2 : o3)));
      if (wbase + k < ccap32) fuse_exact_one(xf, cst[q][kq], sbase + wbase + k, cnt);
    }
    // ... and the blocks its waves flushed mid-sweep (written to the list by
    // this workgroup, visible to it after the barrier above)
    for (int q = 0; q < PF_WAVES; ++q)
      for (unsigned r = 0; r < wxr[q]; ++r) {
        const uint2 bk = xrc[q][r];
        for (unsigned k = threadIdx.x; k < bk.y; k += PF_BLOCK)
          if (bk.x + k < ccap32) fuse_exact_one(xf, ccand[bk.x + k], sbase + bk.x + k, cnt);
      }
  }
#ifdef BSA_PF_STAMPS
  PF_STAMP(3);
  if (lane == 0)
    for (int k = 0; k < 8; ++k) atomicAdd(&cnt->stamp[k], st_acc[k]);
#endif
}


// ------------------------------------------------------------------ single-pass scan
// Exclusive prefix sum of n unsigned words in ONE launch (replaces hipcub's
// three: look-back init + scan, ~16 us per detect at 100k): decoupled
// look-back over 8192-word tiles.  Tiles are numbered by a ticket (a running
// device counter; the host knows its base), so a tile only ever waits on tiles
// that already started.  Tile status words carry the launch's epoch, so they
// need no zeroing between launches: {epoch:30 | flag:2 | value:32}, flag 1 =
// the tile's own total, 2 = inclusive prefix through the tile.
// Tiles of kScanThreads x kScanItems words: 2048 below 2^19 words (more tiles
// in flight: K2 26.3 -> 24.6 us at 100k, 19.9 -> 14.6 us for one rank of 8),
// 8192 above (at 1M a 2048-word tiling's ~1000 tiles lengthened the ticket
// queue and the look-back: 62 -> 139 us)
__device__ __forceinline__ unsigned long long scan_word(unsigned epoch, unsigned flag, unsigned v) {
  return ((unsigned long long)(epoch & 0x3fffffffu) << 34) | ((unsigned long long)flag << 32) | v;
}
template <int kScanThreads, int kScanItems>
__global__ __launch_bounds__(kScanThreads) void k_scan_excl(const unsigned *__restrict__ in, unsigned *__restrict__ out,
                                                            int n, unsigned long long *__restrict__ ticket,
                                                            unsigned long long base,
                                                            unsigned long long *__restrict__ status, unsigned epoch) {
  constexpr int kScanTile = kScanThreads * kScanItems;
  __shared__ unsigned wsum[kScanThreads / 64];
  __shared__ unsigned s_tile, s_excl;
  if (threadIdx.x == 0) s_tile = (unsigned)(atomicAdd(ticket, 1ull) - base);
  __syncthreads();
  const unsigned tile = s_tile;
  const long long i0 = (long long)tile * kScanTile + (long long)threadIdx.x * kScanItems;
  unsigned v[kScanItems], tsum = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (i0 + k < n) ? in[i0 + k] : 0u;
    tsum += v[k];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned x = wave_incl_scan(tsum);
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  // wave 0: tile total, then a wave-wide look-back (64 predecessors per round:
  // the nearest inclusive prefix, plus the aggregates after it)
  if (w == 0) {
    const unsigned wv = lane < kScanThreads / 64 ? wsum[lane] : 0u;
    const unsigned wx = wave_incl_scan(wv);
    if (lane < kScanThreads / 64) wsum[lane] = wx - wv;  // exclusive per-wave offsets
    const unsigned total = __builtin_amdgcn_readlane(wx, 63);
    unsigned excl = 0;
    if (tile == 0) {
      if (lane == 0)
        __hip_atomic_store(&status[0], scan_word(epoch, 2, total), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0)
        __hip_atomic_store(&status[tile], scan_word(epoch, 1, total), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      int top = (int)tile - 1;  // highest predecessor not yet summed
      for (;;) {
        const int j = top - lane;
        unsigned long long st = 0;
        if (j >= 0) st = __hip_atomic_load(&status[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned flag = ((unsigned)(st >> 34) == (epoch & 0x3fffffffu)) ? ((unsigned)(st >> 32) & 3u) : 0u;
        // lanes past tile 0 count as "inclusive 0"
        const bool incl = j < 0 || flag == 2, ready = j < 0 || flag != 0;
        const unsigned long long mi = __ballot(incl), mr = __ballot(ready);
        // first lane (nearest predecessor) holding an inclusive prefix, or 64
        const int fi = mi ? __builtin_ctzll(mi) : 64;
        // every lane up to fi must be ready, else spin on this window
        const unsigned long long need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
        if ((mr & need) != need) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        unsigned part = (lane <= fi && j >= 0) ? (unsigned)st : 0u;
        for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o);
        excl += part;
        if (fi < 64) break;
        top -= 64;
      }
      if (lane == 0)
        __hip_atomic_store(&status[tile], scan_word(epoch, 2, excl + total), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  unsigned run = s_excl + wsum[w] + x - tsum;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (i0 + k < n) out[i0 + k] = run;
    run += v[k];
  }
}

int scan_excl(Ctx *c, const unsigned *in, unsigned *out, int n) {
  if (n <= 0) return 0;
  const bool small = n <= (1 << 19);
  const int kScanTile = small ? 512 * 4 : 1024 * 8;
  const unsigned tiles = (unsigned)((n + kScanTile - 1) / kScanTile);
  const size_t had = c->scan_ws.bytes;
  if (!ensure_keep(c, c->scan_ws, 8 * (size_t)(1 + tiles), "scan tile status")) return -1;
  if (c->scan_ws.bytes != had) c->scan_ready = false;  // grown: the new words are uninitialised
  if (!c->scan_ready) {  // ticket counter and tile status start at 0
    BSA_HIP(c, hipMemsetAsync(c->scan_ws.p, 0, c->scan_ws.bytes, c->stream));
    c->scan_ready = true;
    c->scan_tickets = 0;
    c->scan_epoch = 0;
  }
  const unsigned epoch = ++c->scan_epoch;  // never 0: fresh (zeroed) status words are never ready
  unsigned long long *ws = (unsigned long long *)c->scan_ws.p;
  if (small)
    hipLaunchKernelGGL((k_scan_excl<512, 4>), dim3(tiles), dim3(512), 0, c->stream, in, out, n, ws, c->scan_tickets,
                       ws + 1, epoch);
  else
    hipLaunchKernelGGL((k_scan_excl<1024, 8>), dim3(tiles), dim3(1024), 0, c->stream, in, out, n, ws,
                       c->scan_tickets, ws + 1, epoch);
  BSA_HIP(c, hipGetLastError());
  c->scan_tickets += tiles;
  return 0;
}

// ------------------------------------------------------------------ K1b exact
// flat candidate index space: shard s holds min(count_s, cap / kCandShards)
// candidates; pre[s] = candidates of the shards before s, returns the total
__device__ __forceinline__ unsigned long long cand_prefix(const Counters *cnt, unsigned long long cap,
                                                          unsigned long long *pre) {
  const unsigned long long ccap = cap / kCandShards;
  pre[0] = 0;
#pragma unroll
  for (int q = 0; q < kCandShards; ++q) pre[q + 1] = pre[q] + min(cnt->cshard[q][0], ccap);
  return pre[kCandShards];
}
__device__ __forceinline__ bool cand_overflow(const Counters *cnt, unsigned long long cap) {
  const unsigned long long ccap = cap / kCandShards;
  bool o = cnt->k2_demand != 0;  // a K2 row bucket was full: retried with wider buckets
  o |= cnt->halo_ovf != 0 || cnt->halo_miss != 0;  // halo tiles missing: the step is re-run
  o |= cnt->fuse_ovf != 0;  // fused K1b out of flush records: re-run with K1b's own launch
  o |= cnt->tpr_stale != 0;  // a host-kept tile-pair list that no longer covers the records: re-run, rebuilt
#pragma unroll
  for (int q = 0; q < kCandShards; ++q) o |= cnt->cshard[q][0] > ccap;
  return o;
}


// The next detect's listed items (HeavyArgs): every item whose units took at
// least a threshold is listed (two tiers), its cost word zeroed.  Runs on the
// grid's last lanes (K1b: the lanes past the candidate count; k_rowblk's extra
// blocks when K1b is fused into the prefilter -- in K2's launch, whose lanes
// would have had the time, its code cost K2 +5 us even when skipped).
// Called by every thread of a block (block-uniform trips: it synchronises the
// block).  One returning atomic per tier per BLOCK and trip, the block's
// waves placed by an LDS prefix (one per wave contended on two words: ~350
// at the 100k box, serialised at ~88 per us, were most of k_rowblk's 5.7 us).
constexpr int kHeavyMaxWaves = 16;
__device__ __forceinline__ void heavy_next(const HeavyNext &hn) {
  __shared__ unsigned hcnt[2][kHeavyMaxWaves];
  __shared__ unsigned hbase[2];
  const unsigned long long inear = hn.work[1], m = inear + hn.work[2];
  const unsigned long long nt = (unsigned long long)gridDim.x * blockDim.x;
  const unsigned long long g0 = (unsigned long long)blockIdx.x * blockDim.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = (int)(blockDim.x >> 6);
  // trip j: lane k = nt - 1 - (g0 + t) + j nt; the block's smallest is nt - g0 - blockDim.x + j nt
  for (unsigned long long kb = nt - g0 - blockDim.x; kb < m; kb += nt) {
    const unsigned long long k = kb + (blockDim.x - 1 - threadIdx.x);
    unsigned long long slot = 0;
    int tier = 2;
    if (k < m) {
      slot = k < inear ? k : hn.icap - 1 - (k - inear);
      const unsigned cst = hn.cost[slot];
      hn.cost[slot] = 0u;
      tier = cst >= hn.thresh[0] ? 0 : (cst >= hn.thresh[1] ? 1 : 2);
    }
    const unsigned long long mk0 = __ballot(tier == 0), mk1 = __ballot(tier == 1);
    if (lane == 0) {
      hcnt[0][w] = (unsigned)__popcll(mk0);
      hcnt[1][w] = (unsigned)__popcll(mk1);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      unsigned tot = 0;
      for (int v = 0; v < W; ++v) tot += hcnt[threadIdx.x][v];
      hbase[threadIdx.x] = tot ? atomicAdd(&hn.count[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    if (tier < 2) {
      unsigned off = hbase[tier];
      for (int v = 0; v < w; ++v) off += hcnt[tier][v];
      hn.list[tier][off + lane_prefix(tier == 0 ? mk0 : mk1)] = (unsigned)slot;
      hn.flag[slot] = hn.epoch;
    }
    __syncthreads();  // (hcnt / hbase of the next trip)
  }
}

// Results are stored per candidate (flag, key, payload) rather than appended
// to a shared list: appending needs an atomic with return on ONE counter per
// wave, which serialises at ~88/us (MI355X_MICROARCH 'dequeue') and cost
// ~70 us at 100k.  The per-row counts feed K2's counting sort.
// MODE: kExactRec (stored records), kExactKwik (stored records, KWIK),
// kExactHome (records built from the home-ordered state) -- one kernel per
// mode: with all three paths in one body the register allocation covered the
// union (205 VGPRs, 2 waves per SIMD)
constexpr int kExactRec = 0, kExactKwik = 1, kExactHome = 2;
// Stored-record modes at 3 waves per SIMD (139 VGPRs): at 4 the 128-VGPR cap
// spilled 12 B per lane to scratch inside the fp64 chain, and the dense list's
// ~2 400 working waves fit 3 per SIMD in one round anyway (box100k: 0.1394 ->
// 0.1377 ms per step, A/B 4 x 60 steps)
#ifndef BSA_EXACT_WAVES
#define BSA_EXACT_WAVES 3
#endif
#ifndef BSA_EXACT_HOME_WAVES
#define BSA_EXACT_HOME_WAVES 2
#endif
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == kExactHome ? BSA_EXACT_HOME_WAVES : BSA_EXACT_WAVES, 8))) void k_exact(
    const RowRec *__restrict__ R, const ColRec *__restrict__ C,
    const unsigned *__restrict__ perm_r, const unsigned *__restrict__ perm_c,
    const uint2 *__restrict__ cand, Counters *__restrict__ cnt, SoA6 hs,
    unsigned long long cap, double rpz, double hpz, double tla, int rb, int nrows,
    unsigned char *__restrict__ cflag, double *__restrict__ cpay, unsigned char *__restrict__ inconf,
    unsigned long long *__restrict__ tcpamax_bits, unsigned *__restrict__ rowcnt, uint2 *__restrict__ kb,
    int B,
    unsigned *__restrict__ rctl, const Snap *__restrict__ snap_cur, Snap *__restrict__ snap_build, int nsnap,
    HeavyNext hn) {
  if (hn.cost) heavy_next(hn);  // the next detect's listed items, on the grid's last lanes (idle: past the candidates)
  if (cand_overflow(cnt, cap)) return;  // the caller retries with more room
  if (rctl) {  // reuse: after a build this detect's state becomes the snapshot
    const bool built = rctl[0] != 0;
    const int k0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (built)
      for (int k = k0; k < nsnap; k += gridDim.x * blockDim.x) snap_build[k] = snap_cur[k];
    if (k0 == 0) rctl[1] = built ? 0u : rctl[1] + 1u;
  }
  unsigned long long pre[kCandShards + 1];
  const unsigned long long ncand = cand_prefix(cnt, cap, pre);
  const unsigned long long ccap = cap / kCandShards;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long idx = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
       idx < ncand; idx += stride) {
    int sh = 0;
#pragma unroll
    for (int q = 1; q < kCandShards; ++q) sh += (idx >= pre[q]) ? 1 : 0;
    const uint2 p = cand[(unsigned long long)sh * ccap + (idx - pre[sh])];
    unsigned char flag = 0;
    int row = 0;
    {
      // home mode (perm_r == NULL, the resident sim): rows are the home slice
      // [rb, rb + nrows) of the columns; the key's row is the home row, its
      // column the aircraft index (so K2 orders each row's pairs by index)
      const unsigned oi = perm_r ? perm_r[p.x] : (unsigned)rb + p.x, oj = perm_c[p.y];
      if (perm_r ? oi != oj : oi != p.y) {
        PairResult o;
#ifdef BSA_K1B_NOMATH  // diagnostic build (timing of K1b's memory chain alone; results are wrong)
        {
          const RowRec rr = R[p.x];
          const ColRec cc = C[p.y];
          o = PairResult{false, false, rr.lat, cc.lat, rr.lon, cc.lon, 0.0};
        }
#else
        if (MODE == kExactHome) {  // the records from the state arrays (rows = columns' slice)
          const ColRec ri = col_record(hs, hs, (int)oi), cj = col_record(hs, hs, (int)p.y);
          o = eval_pair<false>(reinterpret_cast<const RowRec &>(ri), cj, rpz, hpz, tla);
        } else {
          o = eval_pair<MODE == kExactKwik>(R[p.x], C[p.y], rpz, hpz, tla);
        }
#endif
#ifdef BSA_K1B_NOATOM  // diagnostic build (K1b without its per-row count atomics; results are wrong)
        {
          double *rq = cpay + idx * kPayStride;
          rq[1] = o.qdr;
          rq[2] = o.dist;
          rq[3] = o.tcpa;
          rq[4] = o.tin;
          rq[5] = o.dcpa + (o.conf ? 1.0 : 0.0) + (o.los ? 2.0 : 0.0);
        }
        o.conf = o.los = false;
#endif
        flag = (o.conf ? 1 : 0) | (o.los ? 2 : 0);
        row = (int)oi - rb;
        if (B) {  // row buckets (k_rank_rows writes inconf / tcpamax per row)
          exact_bucket(o, row, oj, p.y, idx, nrows, B, cpay, rowcnt, kb, cnt);
        } else {
          // one 48-B record per candidate: key | qdr dist tcpa tin dcpa (conflicts)
          double *rec = cpay + idx * kPayStride;
          if (flag) rec[0] = __longlong_as_double((long long)(((unsigned long long)oi << 32) | oj));
          if (o.conf) {
            rec[1] = o.qdr;
            rec[2] = o.dist;
            rec[3] = o.tcpa;
            rec[4] = o.tin;
            rec[5] = o.dcpa;
            inconf[row] = 1;
            // tcpamax = max_j(tcpa * swconfl) >= +-0 (StateBasedCD.py:90): only
            // positive tcpa can raise it, and positive doubles order as integers.
            if (o.tcpa > 0.0)
              atomicMax(&tcpamax_bits[row], (unsigned long long)__double_as_longlong(o.tcpa));
            atomicAdd(&rowcnt[row], 1u);
          }
          if (o.los) atomicAdd(&rowcnt[nrows + 1 + row], 1u);
        }
      }
    }
    if (!B) cflag[idx] = flag;
  }
}

// ------------------------------------------------------------------ K2 canonical order
// Per-row counting sort.  rowcnt holds [conflicts per row | 0 | LoS per row | 0]
// (2 (nrows + 1) words); its exclusive scan rowoff gives each row's segment
// in the conflict list and (minus P) in the LoS list.  k_scatter drops every
// pair's key into its row segment (in any order); k_rank ranks every entry
// among its row segment's columns, so the lists come out exactly in
// np.where's row-major order (StateBasedCD.py:93-95).  All counts are read on
// the device (no host round trip inside a detect), and nothing is written
// when the candidate list overflowed: the caller retries with more room.
__global__ __launch_bounds__(256) void k_scatter(const Counters *__restrict__ cnt, unsigned long long cap,
                                                 int rb, int nrows, const unsigned char *__restrict__ cflag,
                                                 const double *__restrict__ cpay,
                                                 const unsigned *__restrict__ rowoff,
                                                 unsigned *__restrict__ rowcnt,
                                                 unsigned long long *__restrict__ skey,
                                                 unsigned *__restrict__ sslot,
                                                 unsigned long long *__restrict__ lkey) {
  if (cand_overflow(cnt, cap)) return;
  unsigned long long pre[kCandShards + 1];
  const unsigned long long ncand = cand_prefix(cnt, cap, pre);
  const unsigned P = rowoff[nrows];
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long k = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; k < ncand;
       k += stride) {
    const unsigned char f = cflag[k];
    if (!f) continue;
    const unsigned long long key = (unsigned long long)__double_as_longlong(cpay[k * kPayStride]);
    const int row = (int)(key >> 32) - rb;
    if (f & 1) {
      const unsigned pos = rowoff[row] + atomicSub(&rowcnt[row], 1u) - 1u;
      skey[pos] = key;
      sslot[pos] = (unsigned)k;
    }
    if (f & 2) {
      const int r = nrows + 1 + row;
      lkey[rowoff[r] - P + atomicSub(&rowcnt[r], 1u) - 1u] = key;
    }
  }
}

// MVP's per-pair vectors written by k_rank in the resident step (pdv == NULL: off)
struct MvpFuse {
  bsa_mvp_params p;
  MvpPairIn in;
  double4 *pdv;
  uint8_t *pfl;
  double4 *rowdv;  // k_rank_rows: each row's folded dv (mvp_fold), or NULL
};

// One lane per pair slot of the scattered lists (grid-stride over P + L, the
// device-side counts): the slot's rank among its row segment's columns (the
// segment is short: ~1.5 pairs per row at the 100k box; any length works)
// is its final index, so ci / cj / payload (conflicts) and li / lj (LoS)
// come out exactly in np.where's row-major order.  Every lane issues its
// segment loads independently: ~4 dependent memory round trips per detect
// instead of a per-row chain.  Block 0 / lane 0 also publishes the detect's
// totals: cnt->conf / los, the accumulated statistics and the gate words
// (gate[0] = overflow, gate[1] = P) the resident sim step reads.
__global__ __launch_bounds__(256) void k_rank(int nrows, Counters *__restrict__ cnt, unsigned long long cap,
                                              const unsigned *__restrict__ rowoff,
                                              const unsigned long long *__restrict__ skey,
                                              const unsigned *__restrict__ sslot,
                                              const double *__restrict__ cpay,
                                              const unsigned long long *__restrict__ lkey, int rb,
                                              int *__restrict__ ci, int *__restrict__ cj, double *__restrict__ out,
                                              int *__restrict__ li, int *__restrict__ lj,
                                              unsigned long long *__restrict__ stats,
                                              unsigned long long *__restrict__ gate,
                                              const unsigned *__restrict__ build, MvpFuse mf, NfArgs nf,
                                              unsigned long long *__restrict__ tcpamax_bits) {
  const bool ovf = cand_overflow(cnt, cap);
  const bool nfcol = nf.word && *nf.word == nf.epoch;
  const unsigned P = rowoff[nrows], L = rowoff[2 * nrows + 1] - P;
  const unsigned t0 = blockIdx.x * blockDim.x + threadIdx.x;
  if (t0 == 0) {
    unsigned long long pre[kCandShards + 1];
    (void)cand_prefix(cnt, cap, pre);
    unsigned long long ncand = 0;  // candidates written (the prefilter's per-workgroup counts; the list is dense)
    for (int q = 0; q < 32; ++q) ncand += cnt->gpart[q][1];
    cnt->conf = ovf ? 0 : P;
    cnt->los = ovf ? 0 : L;
    cnt->cand = ncand;
    unsigned long long g = 0;
    for (int q = 0; q < 32; ++q) g += cnt->gpart[q][0];
    cnt->groups = g;
    const bool built = !build || build[0];  // a reused list swept nothing this detect
    // an overflowed detect is retried and counted once, when it completes; a
    // list built by a detect whose K2 row buckets overflowed is complete and
    // reused by the retry, so that build counts
    bool list_ovf = false;
    for (int q = 0; q < kCandShards; ++q) list_ovf |= cnt->cshard[q][0] > cap / kCandShards;
    if (built && !list_ovf) {
      stats[0] += cnt->groups;
      stats[2] += cnt->tiles;
      stats[4] += 1;
    }
    if (!ovf) {
      stats[1] += ncand;
      stats[3] += 1;
    }
    if (gate) {
      gate[0] = ovf ? kGateOverflow : (nfcol ? kGateNonfinite : 0);
      gate[1] = ovf ? 0 : P;
      gate[2] = 1ull;  // (HK: no prediction from this K2 form -- rebuild, the safe side)
    }
  }
  if (ovf) return;
  const unsigned stride = gridDim.x * blockDim.x;
  if (nfcol || nf.rowbad)  // non-finite tcpa inputs: tcpamax NaN (K1b's atomics left the others)
    for (int r = (int)t0; r < nrows; r += (int)stride)
      if (nfcol || nf.rowbad[r]) tcpamax_bits[r] = kNanBits;
  for (unsigned x = t0; x < P + L; x += stride) {
    const bool conf = x < P;
    const unsigned long long *keys = conf ? skey : lkey;
    const unsigned xl = conf ? x : x - P;
    const unsigned long long kk = keys[xl];
    const int row = (int)(kk >> 32) - rb;
    const unsigned col = (unsigned)kk;
    const unsigned base = conf ? 0u : P;
    const unsigned b = rowoff[(conf ? 0 : nrows + 1) + row] - base;
    const unsigned e = rowoff[(conf ? 1 : nrows + 2) + row] - base;
    unsigned rank = 0;
    for (unsigned y = b; y < e; ++y) rank += ((unsigned)keys[y] < col) ? 1u : 0u;
    const unsigned pos = b + rank;
    if (conf) {
      const unsigned v = sslot[xl];
      ci[pos] = (int)(kk >> 32);
      cj[pos] = (int)col;
      double pay[5];
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        pay[f] = cpay[(size_t)v * kPayStride + 1 + f];
        out[(size_t)f * P + pos] = pay[f];
      }
      if (mf.pdv) {  // resident step: MVP's per-pair vector (MVP.py:33-56) for k_mvp_row
        double4 dv;
        uint8_t fl;
        mvp_pair(mf.p, mf.in, (int)(kk >> 32), (int)col, pay[0], pay[1], pay[2], pay[3], dv, fl);
        mf.pdv[pos] = dv;
        mf.pfl[pos] = fl;
      }
    } else {
      li[pos] = (int)(kk >> 32);
      lj[pos] = (int)col;
    }
  }
}

// K2 with row buckets (K1b wrote each row's (column, candidate) entries in
// any order and the pair counts of every kRankRows-row block): workgroup b
// takes rows [b kRankRows, (b + 1) kRankRows), one per lane.  Its conflict /
// LoS bases are the block counts before b (and P, the total, for the LoS
// list), its rows' offsets an LDS scan of their counts -- rowoff comes out
// exactly as the scan of the scatter path made it, without a scan launch and
// its look-back chain.  Then the block's pairs, flattened (one lane each):
// the row by binary search over the offsets, the pair's rank among its row's
// bucket (the row's columns) its place in np.where's row-major order
// (StateBasedCD.py:93-95), its payload gathered from its candidate record.
// Block 0 / lane 0 publishes the totals as k_rank does.
// the conflict / LoS pair counts of every kRankRows-row block (behind the
// per-row counts: bcnt[b], bcnt[nb + b]); one wave per block, kRankRows / 64
// rows per lane (one load round trip; an overflowed detect's sums are never
// read: k_rank_rows checks the overflow itself)
// k_rowblk: 16 waves per block, wave w of block b sums row block 16 b + w
constexpr int kRowblkWaves = 16;
constexpr unsigned kHeavyBlocks = 64;  // k_rowblk's extra blocks for the heavy-item listing (65 536 lanes)
__global__ __launch_bounds__(64 * kRowblkWaves) void k_rowblk(int nrows, unsigned *__restrict__ rowcnt, HeavyNext hn) {
  // (K1b fused into the prefilter: the next detect's listed items here, on
  // every lane of the grid -- the host adds kHeavyBlocks blocks past the
  // row-block sums for them, ~1 slot per lane at the 100k box)
  if (hn.cost) heavy_next(hn);
  const int nb = rank_blocks(nrows), b = blockIdx.x * kRowblkWaves + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= nb) return;
  unsigned c = 0, l = 0;
#pragma unroll
  for (int q = 0; q < kRankRows / 64; ++q) {
    const int r = b * kRankRows + q * 64 + lane;
    c += r < nrows ? rowcnt[r] : 0u;
    l += r < nrows ? rowcnt[nrows + 1 + r] : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += (unsigned)__shfl_xor((int)c, o);
    l += (unsigned)__shfl_xor((int)l, o);
  }
  if (lane == 0) {
    rowcnt[2 * (nrows + 1) + b] = c;
    rowcnt[2 * (nrows + 1) + nb + b] = l;
  }
}

template <bool K24>
__global__ __launch_bounds__(kRankThreads) void k_rank_rows(int nrows, Counters *__restrict__ cnt, unsigned long long cap,
                                                         unsigned *__restrict__ rowoff,
                                                         unsigned *__restrict__ rowcnt,
                                                         const uint2 *__restrict__ kb, int B,
                                                         const double *__restrict__ cpay, int rb,
                                                         int *__restrict__ ci, int *__restrict__ cj,
                                                         double *__restrict__ out, int *__restrict__ li,
                                                         int *__restrict__ lj, unsigned long long *__restrict__ stats,
                                                         unsigned long long *__restrict__ gate,
                                                         const unsigned *__restrict__ build, MvpFuse mf,
                                                         unsigned char *__restrict__ inconf,
                                                         unsigned long long *__restrict__ tcpamax_bits,
                                                         Counters *__restrict__ cnext,
                                                         unsigned long long *__restrict__ wnext, K24Args ka,
                                                         NfArgs nf, unsigned long long *__restrict__ hkp) {
  constexpr int W = kRankThreads / 64;
  __shared__ unsigned red[4][W];
  __shared__ unsigned soff[2][kRankRows + 1];  // the block's rows' exclusive offsets (conf, LoS), + total
  // the block's MVP pair vectors for the fold (when they fit; else through pdv / pfl)
  __shared__ double4 sdv[kRankLds];
  __shared__ uint8_t sfl[kRankLds];
  __shared__ double stc[kRankLds];  // ... and their tcpa (tcpamax)
  const int nb = rank_blocks(nrows), b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const unsigned *bcnt = rowcnt + 2 * (nrows + 1);
  const bool rowlane = t < kRankRows;  // lanes past the block's rows only place pairs
  const int r = rowlane ? b * kRankRows + t : nrows;
  const unsigned c = r < nrows ? rowcnt[r] : 0u, l = r < nrows ? rowcnt[nrows + 1 + r] : 0u;
  // non-finite tcpa inputs (NfArgs; loaded with the counts)
  const bool nfcol = nf.word && *nf.word == nf.epoch;
  const unsigned nfrow = nf.rowbad && r < nrows ? nf.rowbad[r] : 0u;
  // the next detect's per-row counts and counters start at zero (its K0z
  // launch is skipped, detect_enqueue): this block's counts are read, the
  // next detect's counter block (cnext / wnext, double-buffered) is idle
  if (r < nrows) {
    rowcnt[r] = 0u;
    rowcnt[nrows + 1 + r] = 0u;
  }
  if (b == 0) {
    constexpr int kWords = (int)(sizeof(Counters) / 8);
    for (int k = t; k < kWords; k += kRankThreads) reinterpret_cast<unsigned long long *>(cnext)[k] = 0ull;
    for (int k = t; k < kWorkShards * kWorkStride; k += kRankThreads) wnext[k] = 0ull;
  }
  const bool ovf = cand_overflow(cnt, cap);
  // P / L = all conflict / LoS pairs, cb / lb = those of the blocks before b
  unsigned P = 0, L = 0, cb = 0, lb = 0;
  for (int q = t; q < nb; q += kRankThreads) {
    const unsigned x = bcnt[q], y = bcnt[nb + q];
    P += x;
    L += y;
    cb += q < b ? x : 0u;
    lb += q < b ? y : 0u;
  }
  {
    unsigned v[4] = {P, L, cb, lb};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      for (int o = 32; o > 0; o >>= 1) v[k] += (unsigned)__shfl_xor((int)v[k], o);
      if (lane == 0) red[k][w] = v[k];
    }
  }
  const unsigned xc = wave_incl_scan(c), xl = wave_incl_scan(l);
  __shared__ unsigned wsum[2][W];
  if (lane == 63) {
    wsum[0][w] = xc;
    wsum[1][w] = xl;
  }
  __syncthreads();
  P = L = cb = lb = 0;
  unsigned wc = 0, wl = 0, tc = 0, tl = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) {
    P += red[0][q];
    L += red[1][q];
    cb += red[2][q];
    lb += red[3][q];
    wc += q < w ? wsum[0][q] : 0u;
    wl += q < w ? wsum[1][q] : 0u;
    tc += wsum[0][q];
    tl += wsum[1][q];
  }
  if (b == 0 && t == 0) {
    unsigned long long ncand = 0;  // candidates written (the prefilter's per-workgroup counts; the list is dense)
    for (int q = 0; q < 32; ++q) ncand += cnt->gpart[q][1];
    cnt->conf = ovf ? 0 : P;
    cnt->los = ovf ? 0 : L;
    cnt->cand = ncand;
    unsigned long long g = 0;
    for (int q = 0; q < 32; ++q) g += cnt->gpart[q][0];
    cnt->groups = g;
    const bool built = !build || build[0];  // a reused list swept nothing this detect
    bool list_ovf = false;  // (see k_rank)
    for (int q = 0; q < kCandShards; ++q) list_ovf |= cnt->cshard[q][0] > cap / kCandShards;
    if (built && !list_ovf) {
      stats[0] += cnt->groups;
      stats[2] += cnt->tiles;
      stats[4] += 1;
    }
    if (!ovf) {
      stats[1] += ncand;
      stats[3] += 1;
    }
    if (gate) {
      gate[0] = ovf ? kGateOverflow : (nfcol ? kGateNonfinite : 0);
      gate[1] = ovf ? 0 : P;
      gate[2] = hkp && *hkp ? 1ull : 0ull;  // HK: this detect's prediction, all-reduced with the gate
    }
    if (hkp) *hkp = 0ull;  // (the word's next writer is two detects on)
    // HK, fused K4' (one rank): this detect's prediction to the host, before
    // any return (the host may be waiting for it); here rather than at the
    // kernel's start, where its loads cost every workgroup ~5 us
    if (K24) hk_publish(ka.pub, [&] { return ovf || *ka.d.sticky != 0u; });
  }
  // fused K4' (K24): an aborted step (this detect overflowed, or an earlier
  // step of the batch did) keeps every row's state -- including the double
  // buffer's other half, which the host swaps in after the step
  const bool k24_stop = K24 && (ovf || *ka.d.sticky != 0u);
  if (K24 && k24_stop) {
    if (ovf && b == 0 && t == 0) ka.mv.sticky[0] = 1u;
    if (rowlane && r < nrows) {
      const int k = rb + r;
      ka.d.alt_w[k] = ka.d.alt[k];
      ka.d.vs_w[k] = ka.d.vs[k];
      ka.d.gse_w[k] = ka.d.gse[k];
      ka.d.gsn_w[k] = ka.d.gsn[k];
    }
    return;
  }
  if (ovf) return;
  const unsigned ec = wc + xc - c, el = wl + xl - l;  // exclusive, within the block
  if (rowlane) {
    soff[0][t] = ec;
    soff[1][t] = el;
  }
  if (t == 0) {
    soff[0][kRankRows] = tc;
    soff[1][kRankRows] = tl;
  }
  if (r < nrows) {
    rowoff[r] = cb + ec;
    rowoff[nrows + 1 + r] = P + lb + el;
  }
  if (b == nb - 1 && t == 0) {
    rowoff[nrows] = P;
    rowoff[2 * nrows + 1] = P + L;
  }
  __syncthreads();
  const bool lds = tc <= (unsigned)kRankLds;  // the block's conflict pairs fit the LDS arrays
  const bool lds_fold = mf.rowdv && lds;
  for (unsigned x = t; x < tc + tl; x += kRankThreads) {
    const bool conf = x < tc;
    const unsigned q = conf ? x : x - tc;
    const unsigned *so = soff[conf ? 0 : 1];
    int lo = 0, hi = kRankRows;  // the last row i with so[i] <= q (rows without pairs share their successor's offset)
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (so[mid] <= q) lo = mid;
      else hi = mid;
    }
    const unsigned k = q - so[lo], m = so[lo + 1] - so[lo];
    const int row = b * kRankRows + lo;
    const uint2 *bk = kb + ((size_t)(conf ? 0 : nrows) + row) * B;
    uint2 e;
    unsigned rank = 0;
    if (B == 8) {  // the whole bucket (one 64-B line, always allocated) in 4 loads issued together,
                   // not one dependent round trip per entry of the row
      uint4 q[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] = reinterpret_cast<const uint4 *>(bk)[u];
      const unsigned col[8] = {q[0].x, q[0].z, q[1].x, q[1].z, q[2].x, q[2].z, q[3].x, q[3].z};
      const unsigned cid[8] = {q[0].y, q[0].w, q[1].y, q[1].w, q[2].y, q[2].w, q[3].y, q[3].w};
      e = make_uint2(0u, 0u);
#pragma unroll
      for (unsigned y = 0; y < 8; ++y)
        if (y == k) e = make_uint2(col[y], cid[y]);
#pragma unroll
      for (unsigned y = 0; y < 8; ++y) rank += (y < m && col[y] < e.x) ? 1u : 0u;
    } else {
      e = bk[k];
      for (unsigned y = 0; y < m; ++y) rank += (bk[y].x < e.x) ? 1u : 0u;
    }
    if (conf) {
      const unsigned pos = cb + so[lo] + rank;
      ci[pos] = rb + row;
      cj[pos] = (int)e.x;
      double pay[5];
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        pay[f] = cpay[(size_t)e.y * kPayStride + 1 + f];
        out[(size_t)f * P + pos] = pay[f];
      }
      const unsigned jh = (unsigned)__double_as_longlong(cpay[(size_t)e.y * kPayStride]);  // (K1b: home column)
      if (lds) stc[so[lo] + rank] = pay[2];
      if (mf.pdv) {  // resident step: MVP's per-pair vector (MVP.py:33-56), folded below
        double4 dv;
        uint8_t fl;
        MvpPairIn in = mf.in;
        int j = (int)e.x;
        if (in.id2h) {  // home order: the intruder's home position as K1b stored it
          j = (int)jh;
          in.id2h = nullptr;
        }
        mvp_pair(mf.p, in, rb + row, j, pay[0], pay[1], pay[2], pay[3], dv, fl);
        if (lds_fold) {
          sdv[so[lo] + rank] = dv;
          sfl[so[lo] + rank] = fl;
        } else {
          mf.pdv[pos] = dv;
          mf.pfl[pos] = fl;
        }
      }
    } else {
      const unsigned pos = lb + so[lo] + rank;
      li[pos] = rb + row;
      lj[pos] = (int)e.x;
    }
  }
  // per row (this workgroup's stores are visible to its lanes after the
  // barrier): inconf = any conflict (StateBasedCD.py:89), tcpamax =
  // max_j(tcpa * swconfl) (:90) -- +0 or the largest positive tcpa, as K1b's
  // atomics on the bit patterns made it -- and K3's fold of the row's pairs,
  // in order (MVP.py:44-61), from LDS or from pdv / pfl
  __syncthreads();
  const bool live = rowlane && r < nrows;
  if (!K24 && !live) return;
  if (live) {
    inconf[r] = c ? 1 : 0;
    unsigned long long tm = 0ull;
    for (unsigned k = 0; k < c; ++k) {
      const double tq = lds ? stc[ec + k] : out[(size_t)2 * P + cb + ec + k];
      const unsigned long long bits = (unsigned long long)__double_as_longlong(tq);
      if (tq > 0.0 && bits > tm) tm = bits;
    }
    // non-finite tcpa inputs in some column (every row) or in this row: NaN,
    // as np.max propagates it
    tcpamax_bits[r] = nfcol || nfrow ? kNanBits : tm;
    if (mf.rowdv)
      mf.rowdv[r] = lds_fold ? mvp_fold(sdv, sfl, ec, ec + c) : mvp_fold(mf.pdv, mf.pfl, cb + ec, cb + ec + c);
  }
  if (K24) {  // K4' of this workgroup's rows (k_sim_pilot_kin<true, PREP>'s body), every lane
    __shared__ unsigned long long sgate[2];
    if (t == 0) {
      sgate[0] = 0ull;
      sgate[1] = P;
    }
    __syncthreads();
    if (b == 0 && t == 0) *ka.d.steps_done += 1;
    MvpIn mv = ka.mv;
    mv.gate = sgate;
    const int k = rb + r;  // (rows = all aircraft: rb = 0)
    // the wave's group boxes from its lanes' records (lanes past nrows too, whose zeroed
    // records reduce to nothing); waves past the block's rows (BSA_RANK_LANES_PER_ROW > 1)
    // hold no rows and must not write a box (wave-uniform: kRankRows % 64 == 0)
    if (ka.prep && rowlane) {
      PFRec pr{}, pb{};
      if (ka.pa.snap && live) pb = ka.pa.snap[k];
      if (live)
        pr = pilot_kin_row<true, true>(rb, k, ka.simdt, ka.winddim, ka.vwn, ka.vwe, ka.wf, ka.d, mv, ka.mp, ka.pa);
      group_boxes_v(ka.pa.n, k / kGroup, pr, ka.pa.sbox, ka.pa.gbox);
      if (ka.pa.snap) {
        const bool outb = live && !pf_within(pr, pb, ka.pa.dx, ka.pa.ds, ka.pa.dv);
        if (__ballot(outb) && lane == 0) ka.pa.tpr_ctl[0] = 1ull;
        if (ka.pa.pred) {  // HK: ... or f x the budgets (a rebuild two detects on)
          const float f = ka.pa.pf;
          const bool nearb = live && !pf_within(pr, pb, f * ka.pa.dx, f * ka.pa.ds, f * ka.pa.dv);
          if (__ballot(nearb) && lane == 0) *ka.pa.pred = 1ull;
        }
      }
    } else if (live) {
      pilot_kin_row<true, false>(rb, k, ka.simdt, ka.winddim, ka.vwn, ka.vwe, ka.wf, ka.d, mv, ka.mp, ka.pa);
    }
  }
}

// Zero the per-detect state: counters (but `tiles` unless full; with keep,
// nothing of the candidate list: its counts, tiles and groups), the dequeue
// shards and the per-row outputs / counts.  Grid-stride, one word per lane
// (zero_state, shared with the fused K0z+K0b path of k_prep_cols).
// tbox (nullable): the tile boxes of cnt records from their group boxes (the
// records and group boxes were written by the resident step's K4').
__global__ __launch_bounds__(256) void k_zero(int nrows, int full, int keep, unsigned *__restrict__ rctl,
                                              int rforce, Counters *__restrict__ cnt,
                                              unsigned long long *__restrict__ work,
                                              unsigned char *__restrict__ inconf,
                                              unsigned long long *__restrict__ tcpamax,
                                              unsigned *__restrict__ rowcnt, int tcnt,
                                              const TileBox *__restrict__ gbox, TileBox *__restrict__ tbox) {
  if (rctl && blockIdx.x == 0 && threadIdx.x == 0) {  // reuse: build this detect? (force: age 0)
    rctl[0] = rforce ? 1u : 0u;
    if (rforce) rctl[1] = 0u;
  }
  if (tbox)
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < (tcnt + kTile - 1) / kTile; t += gridDim.x * blockDim.x)
      tile_from_groups(tcnt, t, gbox, tbox);
  zero_state(ZeroArgs{nrows, full, keep, cnt, work, inconf, tcpamax, rowcnt, {}, {}},
             blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// ------------------------------------------------------------------ host side
static inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// spatial sort of cnt positions starting at original index base -> perm
static int spatial_order(Ctx *c, int cnt, int base, const double *lat, const double *lon, const double *trk,
                         const double *gs, double f, DevBuf &key, DevBuf &idx, DevBuf &key2, DevBuf &perm) {
  if (!ensure(c, key, (size_t)cnt * 4, "keys") || !ensure(c, idx, (size_t)cnt * 4, "key idx") ||
      !ensure(c, key2, (size_t)cnt * 4, "sorted keys") || !ensure(c, perm, (size_t)cnt * 4, "perm"))
    return -1;
  hipLaunchKernelGGL(k_keys, dim3(blocks_for(cnt, 256)), dim3(256), 0, c->stream, cnt, base, lat, lon, trk, gs,
                     f, (unsigned *)key.p, (unsigned *)idx.p);
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

// Home order of the resident sim (bsa_sim_init): the spatial order of the
// traffic in own[] (aircraft-index order) at the look-ahead midpoints the
// detect's stage 1 uses -> h2id (home position -> aircraft index).  Every rank
// computes the same permutation from the same state (deterministic sort).
int home_order(Ctx *c, double tla, std::vector<unsigned> &h2id) {
  const int64_t n = c->n;
  const double kf = 0.5 * (tla > 0.0 ? tla : 0.0) / 6371000.0;
  DevBuf key, idx, key2, perm;
  struct Rel {
    DevBuf *b[4];
    ~Rel() {
      for (auto *x : b) release(*x);
    }
  } rel{{&key, &idx, &key2, &perm}};
  if (spatial_order(c, (int)n, 0, (const double *)c->own[0].p, (const double *)c->own[1].p,
                    (const double *)c->own[2].p, (const double *)c->own[3].p, kf, key, idx, key2, perm))
    return -1;
  h2id.assign((size_t)n, 0u);
  BSA_HIP(c, hipMemcpyAsync(h2id.data(), perm.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// event set of this detect (the pool keeps one set per detect since the last
// bsa_timing_reset, up to kEvSets; later detects reuse the last set)
static int next_events(Ctx *c, hipEvent_t **ev) {
  const int k = std::min(c->ev_sets, kEvSets - 1);
  if ((int)c->evpool.size() < 5 * (k + 1)) {
    const size_t old = c->evpool.size();
    c->evpool.resize(5 * (size_t)(k + 1), nullptr);
    // timing-only events: no system-scope fence at record (a fenced record left a
    // ~6 us bubble before the next kernel, 5 per detect; only elapsed times are read)
    for (size_t q = old; q < c->evpool.size(); ++q)
      BSA_HIP(c, hipEventCreateWithFlags(&c->evpool[q], hipEventDisableSystemFence));
  }
  *ev = &c->evpool[5 * (size_t)k];
  c->ev_last = k;
  if (c->ev_sets < kEvSets) c->ev_sets++;
  return 0;
}

// stage 1 at the look-ahead midpoints unless KWIK, candidate
// reuse, BSA_FLAG_STAGE1_T0 or the BSA_STAGE1_T0 environment variable
// home mode: K1b reads stored fp64 column records (else builds them from the
// state arrays); BSA_HOME_REC=0/1 overrides (see detect_enqueue)
// One rank below 163 840 rows stores them (K1b then runs fused into the
// prefilter, on stored records; 500k and 1M rows are slower with them).  A
// rank of a row-sharded step (halo mode) does not: its two K0b launches (own
// and halo tiles) would write 128 B per column, and its K1b runs unfused
// anyway.  Measured with the whole rank step (tools/probe_step.py, 200 settle
// steps, slowest rank, BSA_HOME_REC=1 -> 0, A/B x 2): global1m R = 8 0.1175 /
// 0.1175 -> 0.1115 / 0.1127 ms, box100k R = 8 0.0822 / 0.0827 -> 0.0806 /
// 0.0800, R = 4 0.0966 / 0.0974 -> 0.0945 / 0.0939, R = 2 0.1092 / 0.1088 ->
// 0.1109 / 0.1082 (an older detect-only probe with per-stage events had
// favoured the records by ~4 us).
bool home_records(const Ctx *c, int64_t nrows) {
  static const int home_rec_env = getenv("BSA_HOME_REC") ? atoi(getenv("BSA_HOME_REC")) : -1;
  return home_rec_env >= 0 ? home_rec_env == 1 : c->halo_mode == 0 && nrows <= 163840;
}

int stage1_mid(int flags, bool reuse, int kwik) {
  static const bool t0_env = getenv("BSA_STAGE1_T0") && atoi(getenv("BSA_STAGE1_T0")) != 0;
  return (!reuse && !kwik && !(flags & BSA_FLAG_STAGE1_T0) && !t0_env) ? 1 : 0;
}

static SoA6 soa(const DevBuf *a) {
  return SoA6{(const double *)a[0].p, (const double *)a[1].p, (const double *)a[2].p,
              (const double *)a[3].p, (const double *)a[4].p, (const double *)a[5].p};
}

int prep_all_tiles(Ctx *c, double rpz, double hpz, double tla, unsigned long long nf_epoch) {
  const int64_t n = c->n;
  if (n <= 0) return 0;
  const int nct = (int)((n + kTile - 1) / kTile);
  if (!ensure(c, c->colrec, n * sizeof(ColRec), "column records") ||
      !ensure(c, c->pfcol, n * sizeof(PFRec), "prefilter columns") ||
      !ensure(c, c->pfvcol, n * sizeof(PFVel), "prefilter column velocities") ||
      !ensure(c, c->pfpcol, n * sizeof(float4), "prefilter column positions") ||
      !ensure(c, c->tbox_c, nct * sizeof(TileBox), "column tile boxes") ||
      !ensure(c, c->gbox_c, ((n + kGroup - 1) / kGroup) * sizeof(TileBox), "column group boxes") ||
      !ensure(c, c->sbox_c, ((n + kSub - 1) / kSub) * sizeof(TileBox), "column sub-group boxes"))
    return -1;
  const SoA6 own = soa(c->own);
  const FusedBoxes fb{(TileBox *)c->sbox_c.p, (TileBox *)c->gbox_c.p, (TileBox *)c->tbox_c.p, nullptr, 0};
  const ZeroArgs zs{0, 1, 0, nullptr, nullptr, nullptr, nullptr, nullptr, {}, {}};
  hipLaunchKernelGGL(k_prep_cols, dim3((unsigned)nct), dim3(kTile), 0, c->stream, (int)n,
                     (const unsigned *)c->h2id.p, 1, 0, own, own, 0, 1, rpz, hpz, tla, (ColRec *)c->colrec.p,
                     (PFRec *)c->pfcol.p, (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, stage1_mid(0, false, 0),
                     ReuseParams{}, fb, zs, 0, (const int *)nullptr, HaloUnpack{}, (Counters *)nullptr, TprCheck{},
                     NfArgs{nf_epoch ? (unsigned long long *)c->nonfin.p : nullptr, nf_epoch, nullptr}, nct);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

// Enqueue one complete detect on the stream (K0-K2), no host synchronisation.
// gate (device, nullable): receives {overflow, P} for the resident sim step.
// k_rank_rows' arguments (kept for a fused launch, k24_launch)
struct RankLaunch {
  unsigned grid;
  int nrows;
  Counters *cnt;
  unsigned long long cap;
  unsigned *rowoff, *rowcnt;
  const uint2 *kb;
  int B;
  const double *cpay;
  int rb;
  int *ci, *cj;
  double *out;
  int *li, *lj;
  unsigned long long *stats, *gate;
  const unsigned *build;
  MvpFuse mf;
  unsigned char *inconf;
  unsigned long long *tcpamax;
  Counters *cnext;
  unsigned long long *wnext;
  NfArgs nf;
  unsigned long long *hkp;  // HK: the prediction word K2 moves into gate[2] (NULL: none / fused K4' publishes it)
};
static int rank_launch(Ctx *c, const RankLaunch &a, bool k24, const K24Args &ka) {
  const auto K = k24 ? k_rank_rows<true> : k_rank_rows<false>;
  hipLaunchKernelGGL(K, dim3(a.grid), dim3(kRankThreads), 0, c->stream, a.nrows, a.cnt, a.cap, a.rowoff, a.rowcnt,
                     a.kb, a.B, a.cpay, a.rb, a.ci, a.cj, a.out, a.li, a.lj, a.stats, a.gate, a.build, a.mf,
                     a.inconf, a.tcpamax, a.cnext, a.wnext, ka, a.nf, k24 ? nullptr : a.hkp);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

bool nonfin_word(Ctx *c) {
  const bool fresh = !c->nonfin.p;
  if (!ensure(c, c->nonfin, 16, "non-finite input word")) return false;
  if (fresh && hipMemsetAsync(c->nonfin.p, 0, 16, c->stream) != hipSuccess) {
    fail(c, "zeroing the non-finite input word failed");
    return false;
  }
  return true;
}

// HK: wait until the step of detect m published its prediction (ring slot m
// % kHkRing holds (m + 1) << 2 | flags); the device runs the step before the
// one being enqueued, so this normally returns at once or after part of a step
static int hk_wait(Ctx *c, int64_t m, unsigned long long *v) {
  volatile unsigned long long *p = c->hk_host + (m % kHkRing);
  const unsigned long long want = (unsigned long long)(m + 1);
  if ((*p >> 2) == want) {
    *v = *p;
    return 0;
  }
  c->hk_waits++;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; ++spin) {
    const unsigned long long x = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    if ((x >> 2) == want) {
      *v = x;
      return 0;
    }
    if ((spin & 1023u) == 1023u) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
        return fail(c, "HK: the device did not publish detect %lld's prediction within 60 s", (long long)m);
      std::this_thread::yield();
    }
  }
}

// the halo overlap's second stream and events (Ctx::ov_*), created once
static int ov_init(Ctx *c) {
  if (!c->xstream) BSA_HIP(c, hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking));
  for (hipEvent_t &e : c->ov_ev)
    if (!e) BSA_HIP(c, hipEventCreateWithFlags(&e, c->ov_evflags));
  return 0;
}

int detect_enqueue(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
                   unsigned long long *gate) {
  c->fuse_done = false;  // set again only if K2 below evaluates MVP's per-pair vectors
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
      !ensure(c, c->counters2, sizeof(Counters), "next counters") ||
      !ensure(c, c->workq2, kWorkShards * kWorkStride * 8, "next work counters") ||
      !ensure(c, c->stats, 8 * 8, "detect statistics") ||
      !ensure(c, c->inconf, (size_t)(nrows > 0 ? nrows : 1), "inconf") ||
      !ensure(c, c->tcpamax, (size_t)(nrows > 0 ? nrows : 1) * 8, "tcpamax") ||
      !ensure(c, c->workq, kWorkShards * kWorkStride * 8, "work counters") ||
      !ensure(c, c->rowcnt, (size_t)rowcnt_words((int)nrows) * 4, "row counts") ||
      !ensure(c, c->rowoff, (size_t)(2 * (nrows + 1)) * 4, "row offsets"))
    return -1;
  const bool distinct = c->has_intruder;
  // home mode (the resident sim, bsa_sim.hip): own[] is already in spatial
  // (home) order, h2id names the aircraft; the rows are the 512-aligned home
  // slice [rb, re) of the columns (no re-sort, no gather)
  const bool home = c->det_home;
  c->last_home = home;
  // halo mode (home mode of the row-sharded step, or its one-GPU probe): K0
  // prepares the rank's own column tiles [a0, a1), halo_mid plans / exchanges
  // the tiles its rows can reach, K0 prepares those from the list
  const bool halo = home && c->halo_mode != 0;
  const int a0 = (int)(rb / kTile), a1 = (int)((re + kTile - 1) / kTile);
  // home mode: K1b builds its fp64 records from the state arrays instead of
  // reading 128-B records K0b wrote for EVERY column: cheaper when K0b's
  // record writes dominate -- at 1M (0.165 -> 0.084 ms of K0) or for one rank's
  // slice of several; with one rank below 2^18 aircraft the stored records
  // win (each aircraft is in ~5 candidates there: K1b 27 -> 18 us at 100k).
  // BSA_HOME_REC=0/1 overrides.
  const bool recs = !home || home_records(c, nrows);
  if (home && (distinct || (rb % kTile != 0 && re > rb) || (flags & BSA_FLAG_KWIK)))  // (a rank without rows: rb = n)
    return fail(c, "home-order detect needs own == intruder, a %d-aligned row slice, no KWIK", kTile);
  const int kwik = (flags & BSA_FLAG_KWIK) ? 1 : 0;
  // KWIK: stage 1 is exact-safe only with the pair's own mean latitude in
  // cavelat (own == intruder), and the CPA refine's geometry
  // is the great circle's: a distinct intruder set disables the prefilter,
  // and the refine keeps every stage-1 survivor.
  const int noprune = ((flags & BSA_FLAG_NOPRUNE) || (kwik && distinct)) ? 1 : 0;
  // rows share the column order and records when own == intruder and the
  // whole range is detected; only then can the candidate list be reused
  const bool shared = home || (!distinct && rb == 0 && re == n);
  const int64_t roff = home ? rb : 0;  // the rows' offset in the shared records
  const bool reuse = c->reuse_on && shared && rb == 0 && re == n && !noprune && !kwik && n > 0 && !halo;
  if (!reuse) c->reuse_valid = false;
  // stage 1 at the look-ahead midpoints: its bound is derived
  // for the great-circle geometry and fixed reaches, so not with KWIK nor with
  // the reuse budgets (whose drift checks assume t = 0 points); the
  // BSA_STAGE1_T0 environment variable selects t = 0 for A/B measurements
  const int mid = stage1_mid(flags, reuse, kwik);
  // the resident step's K4' already wrote this detect's column records and
  // boxes from the state it computed (Ctx::sim_prepped; any detect consumes or
  // invalidates them: it rewrites the same buffers)
  const bool prepped = c->sim_prepped && home && !halo && !reuse && rb == 0 && re == n && flags == 0 &&
                       c->sim_prep_key[0] == rpz && c->sim_prep_key[1] == hpz && c->sim_prep_key[2] == tla &&
                       c->sim_prep_key[3] == (double)mid && c->sim_prep_n == n;
  c->sim_prepped = false;
  // non-finite tcpa inputs: this detect's epoch (the prepped records carry K4''s)
  if (!nonfin_word(c)) return -1;
  NfArgs nfa{(unsigned long long *)c->nonfin.p,
             prepped ? c->nf_prep_epoch : (c->nf_force_epoch ? c->nf_force_epoch : ++c->nf_counter), nullptr};
  // K0z skipped: the last detect's K2 (k_rank_rows) zeroed this detect's
  // counter block (double-buffered), dequeue words and per-row counts, and
  // writes inconf / tcpamax of every row itself; the prepped tile boxes are
  // derived from the group boxes by K0d (direct form only)
  static const bool tp_super = getenv("BSA_TP_SUPER") && atoi(getenv("BSA_TP_SUPER")) == 1;  // (A/B)
  static const bool zero_env = getenv("BSA_K0Z") && atoi(getenv("BSA_K0Z")) == 1;           // (A/B)
  // ---- tile-pair list reuse: the resident step's detects of
  // a rank's rows -- one rank: records prepared (and checked) by K4'; several
  // ranks or the probe: the halo plan is kept with the list.  Any other detect
  // of this context invalidates the kept list.  Halo mode: K0d sweeps the
  // present column tiles only (own + received, the flat halo list;
  // BSA_TP_HALO_ALL=1 sweeps all tiles for A/B).
  static const bool tp_all = getenv("BSA_TP_HALO_ALL") && atoi(getenv("BSA_TP_HALO_ALL")) == 1;
  const bool tp_list = halo && !tp_all && !tp_super;
  static const bool tpr_env = !(getenv("BSA_TPR") && atoi(getenv("BSA_TPR")) == 0);
  const bool tpr = tpr_env && c->tpr_on && home && !reuse && flags == 0 && !tp_super &&
                   ((!halo && prepped && (n + kTile - 1) / kTile <= kTPDirectMax) || tp_list);
  const double tkey[6] = {rpz, hpz, tla, (double)mid, (double)rb, (double)re};
  const bool tvalid = tpr && c->tpr_valid && c->tpr_n == n && memcmp(tkey, c->tpr_key, sizeof tkey) == 0;
  // Who decides a rebuild.  HK (the resident step, Ctx::hk_*): the host, before
  // enqueuing -- a kept list then launches no K0d and, several ranks, no box
  // all-gather, no halo plan and one K0b for own + halo tiles.  Every rank
  // takes the same decision from the same inputs (the host-side invalidations
  // are collective events, the prediction is all-reduced with the gate).
  // Otherwise the device: the records' preparers raise a flag, K0d / the plan
  // read it (round-5 behaviour).
  bool hk = false, hkeep = false;
  int64_t hm = 0;
  if (tpr && c->hk_req && c->hk_on && !c->simp.resume_nav && c->hk_hdev) {
    if (c->hk_cool > 0) {  // after a stale abort: device-decided for a while
      c->hk_cool--;
      c->hk_ok = false;
    } else {
      hk = true;
      hm = c->hk_m++;
      const int nf = (c->simp.winddim == 0 && c->sim_gs_derivable) ? 6 : 8;  // (halo_mid's field count)
      bool build = !tvalid || !c->hk_ok || (c->halo_mode == 1 && nf != c->halo_fields);
      // a build one or two detects ago: its snapshot is fresh enough (the
      // prediction covers two steps of drift); else the prediction made from
      // the records of detect hm - 2, published by that step's K4'
      if (!build && !c->hk_built[(hm + 3) & 3] && !c->hk_built[(hm + 2) & 3]) {
        unsigned long long v = 0;
        if (hk_wait(c, hm - 2, &v)) return -1;
        build = (v & 3ull) != 0;  // predicted, or that step aborted (its retry rebuilds anyway)
      }
      c->hk_built[hm & 3] = build;
      c->hk_ok = true;
      hkeep = !build;
      (build ? c->hk_builds : c->hk_keeps)++;
      static const bool trace = getenv("BSA_HK_TRACE") && atoi(getenv("BSA_HK_TRACE")) == 1;  // (diagnostics)
      if (trace)
        fprintf(stderr, "[bsa hk] rank %d detect %lld: %s (tvalid %d, step %lld)\n", c->rank, (long long)hm,
                build ? "build" : "keep", tvalid ? 1 : 0, (long long)c->sim_steps);
    }
  } else if (tpr) {
    c->hk_ok = false;  // a device-decided detect: the build history is no longer the host's
  }
  c->hk_cur = hk;
  c->hk_keep = hkeep;
  c->hk_last = hm;
  if (tpr) {  // (every rank, also one without rows: the kept state stays collective)
    c->tpr_valid = true;  // (an aborted step or any state change clears it)
    memcpy(c->tpr_key, tkey, sizeof tkey);
    c->tpr_n = n;
  } else {
    c->tpr_valid = false;
  }
  // (HK keep, halo mode: K2 zeroed this detect's counters too, or K0z runs as
  // its own launch -- not inside the merged K0b, whose halo workgroups write Counters)
  const bool nozero = ((prepped && (n + kTile - 1) / kTile <= kTPDirectMax) || (hkeep && halo)) && !zero_env &&
                      !tp_super && c->k2_bucket > 0 && c->zeroed_rows == nrows;
  c->zeroed_rows = -1;
  if (nozero) {
    std::swap(c->counters, c->counters2);
    std::swap(c->workq, c->workq2);
  }
  // stage events of this detect: only one detect in ev_every is timed (each
  // record costs a ~5 us bubble before the next kernel, bsa_set_timing_sample)
  hipEvent_t *ev = nullptr;
  const bool timed = c->ev_every > 0 && (c->ev_count++ % c->ev_every) == 0;
  if (timed && next_events(c, &ev)) return -1;
  auto mark = [&](int e) -> int {
    if (timed) BSA_HIP(c, hipEventRecord(ev[e], c->stream));
    return 0;
  };
  if (mark(0)) return -1;
  Counters *dcnt = (Counters *)c->counters.p;
  // K0z: zero the per-detect state (launched once the reuse decision is known)
  auto zero = [&](bool keep, unsigned *rctl, int rforce, bool tiles = false) -> int {
    const int64_t m = std::max<int64_t>(2 * (nrows + 1), 256);
    hipLaunchKernelGGL(k_zero, dim3((unsigned)std::min<int64_t>(blocks_for(m, 256 * 4), 256)), dim3(256), 0,
                       c->stream, (int)nrows, 1, keep ? 1 : 0, rctl, rforce, dcnt,
                       (unsigned long long *)c->workq.p, (unsigned char *)c->inconf.p,
                       (unsigned long long *)c->tcpamax.p, (unsigned *)c->rowcnt.p, (int)n,
                       (const TileBox *)c->gbox_c.p, tiles ? (TileBox *)c->tbox_c.p : (TileBox *)nullptr);
    BSA_HIP(c, hipGetLastError());
    return 0;
  };
  if (n == 0 || nrows == 0) {
    if (zero(false, nullptr, 0)) return -1;
    if (halo) {  // a rank without rows still takes part in the exchange (HK keep: no box all-gather)
      HaloPre hp;
      HaloUnpack hu;
      if (halo_pre(c, rb, re, &hp)) return -1;
      if (!hkeep) {
        for (int r = 0; r < 3; ++r)
          if (hp.zn[r]) BSA_HIP(c, hipMemsetAsync(hp.z[r], 0, (size_t)hp.zn[r] * 4, c->stream));
        // (its plan-reuse flag stays clear: it holds no records that could drift)
        if (unsigned *f = halo_flag_word(c)) BSA_HIP(c, hipMemsetAsync(f, 0, 4, c->stream));
      }
      if (halo_mid(c, rb, re, &hu, nullptr, hkeep)) return -1;
    }
    if (gate) BSA_HIP(c, hipMemsetAsync(gate, 0, kGateWords * 8, c->stream));
    for (int e = 1; e < 5; ++e)
      if (mark(e)) return -1;
    c->ev_valid = c->ev_valid || timed;
    c->empty_detect = true;
    return 0;
  }
  c->empty_detect = false;
  DevBuf *I = distinct ? c->intr : c->own;
  SoA6 own{(const double *)c->own[0].p, (const double *)c->own[1].p, (const double *)c->own[2].p,
           (const double *)c->own[3].p, (const double *)c->own[4].p, (const double *)c->own[5].p};
  SoA6 intr{(const double *)I[0].p, (const double *)I[1].p, (const double *)I[2].p,
            (const double *)I[3].p, (const double *)I[4].p, (const double *)I[5].p};

  // ---- K0a spatial order.  Any permutation gives identical results (the
  // output is re-sorted canonically), so the order is reused for up to
  // kResortEvery calls on the same shape: aircraft move ~km between calls,
  // tiles span ~100 km (with a reusable list: 64 calls, and every re-sort
  // rebuilds the list).
  const double kf = mid ? 0.5 * (tla > 0.0 ? tla : 0.0) / 6371000.0 : 0.0;  // k_keys midpoint factor
  const bool resort = !home && (!c->perm_valid || c->perm_n != n || c->perm_rb != rb || c->perm_re != re ||
                      c->perm_shared != shared || c->perm_distinct != distinct || c->perm_f != kf ||
                      (flags & BSA_FLAG_RESORT) || c->perm_age >= (reuse ? kResortEveryReuse : kResortEvery));
  // ---- candidate-list reuse: the list of the last build stays valid for
  // this perm / parameters / buffers unless an aircraft overran its budget
  // (decided on the device by K0b; ctl[0] = build this detect)
  if (c->cand_cap == 0)
    // 8 x max(128 k, 4 rows) candidates in all (at 100k rows ~12x the demand), whole shards
    c->cand_cap = (unsigned long long)kCandShards *
                  (((unsigned long long)8 * std::max<int64_t>(1 << 17, 4 * nrows) + kCandShards - 1) / kCandShards);
  const unsigned long long cap = c->cand_cap;
  if (!ensure(c, c->cand, cap * sizeof(uint2), "candidate pairs")) return -1;
  ReuseParams rz{};
  bool rvalid = false;
  if (reuse) {
    if (!ensure(c, c->snap_build, (size_t)n * sizeof(Snap), "reuse snapshot") ||
        !ensure(c, c->snap_cur, (size_t)n * sizeof(Snap), "reuse state") ||
        !ensure(c, c->reuse_use, (size_t)((n + 63) / 64) * 8, "reuse budget use") ||
        !ensure(c, c->reuse_ctl, 16, "reuse control"))
      return -1;
    const double key[4] = {rpz, hpz, tla, (double)flags};
    rvalid = c->reuse_valid && !resort && c->reuse_n == n && c->reuse_cap == cap &&
             c->reuse_candp == c->cand.p && memcmp(key, c->reuse_key, sizeof key) == 0;
    rz.build = (const Snap *)c->snap_build.p;
    rz.cur = (Snap *)c->snap_cur.p;
    rz.ctl = (unsigned *)c->reuse_ctl.p;
    rz.use = (float *)c->reuse_use.p;
    rz.sh = c->reuse_sh;
    rz.sh_chord = (float)(c->reuse_sh / 6.3e6) * 1.000001f;
    rz.sv_default = c->reuse_sv;
    rz.sv_min = 1.0;
    rz.sv_max = 4.0 * c->reuse_sv;
    rz.ktarget = 16.0;
    rz.valid = rvalid ? 1 : 0;
    c->reuse_valid = true;  // optimistic: an overflow invalidates it (detect_finish / sim retry)
    memcpy(c->reuse_key, key, sizeof key);
    c->reuse_n = n;
    c->reuse_cap = cap;
    c->reuse_candp = c->cand.p;
  }
  const unsigned *build = reuse ? (const unsigned *)c->reuse_ctl.p : nullptr;
  // K0z runs inside K0b (k_prep_cols) unless the list is reused (its build flag is set here)
  if (reuse && zero(true, (unsigned *)c->reuse_ctl.p, rvalid ? 0 : 1)) return -1;
  if (resort) {
    // columns: intruder position, own velocity; rows: own position, intruder velocity
    if (spatial_order(c, (int)n, 0, intr.lat, intr.lon, own.trk, own.gs, kf, c->key_c, c->idx_c, c->key_c2,
                      c->perm_c))
      return -1;
    if (!shared && spatial_order(c, (int)nrows, (int)rb, own.lat, own.lon, intr.trk, intr.gs, kf, c->key_r,
                                 c->idx_r, c->key_r2, c->perm_r))
      return -1;
    c->perm_f = kf;
    c->perm_valid = true;
    c->perm_n = n;
    c->perm_rb = rb;
    c->perm_re = re;
    c->perm_shared = shared;
    c->perm_distinct = distinct;
    c->perm_age = 0;
  }
  if (!home) c->perm_age++;
  const unsigned *perm_c = (const unsigned *)(home ? c->h2id.p : c->perm_c.p);
  const unsigned *perm_r = home ? nullptr : (const unsigned *)(shared ? c->perm_c.p : c->perm_r.p);

  // ---- buffers sized by the candidate capacity (every pair list <= candidates)
  if (!ensure(c, c->cflag, cap, "candidate flags") ||
      !ensure(c, c->cpay, cap * kPayStride * 8, "candidate records") ||
      !ensure(c, c->ckey2, cap * 8, "conflict keys") || !ensure(c, c->cval2, cap * 4, "conflict slots") ||
      !ensure(c, c->lkey2, cap * 8, "los keys") || !ensure(c, c->out_ci, cap * 4, "ci") ||
      !ensure(c, c->out_cj, cap * 4, "cj") || !ensure(c, c->out_pay, cap * 5 * 8, "conflict outputs") ||
      !ensure(c, c->out_li, cap * 4, "li") || !ensure(c, c->out_lj, cap * 4, "lj"))
    return -1;
  // ---- K0b records in sorted order (shared: the column records serve as
  // row records too; RowRec and ColRec agree field for field up to `vs`)
  if (!ensure(c, c->colrec, n * sizeof(ColRec), "column records") ||
      !ensure(c, c->pfcol, n * sizeof(PFRec), "prefilter columns") ||
      !ensure(c, c->pfvcol, n * sizeof(PFVel), "prefilter column velocities") ||
      !ensure(c, c->pfpcol, n * sizeof(float4), "prefilter column positions"))
    return -1;
  if (!shared && (!ensure(c, c->rowrec, nrows * sizeof(RowRec), "row records") ||
                  !ensure(c, c->pfrow, nrows * sizeof(PFRec), "prefilter rows") ||
                  !ensure(c, c->pfvrow, nrows * sizeof(PFVel), "prefilter row velocities") ||
                  !ensure(c, c->pfprow, nrows * sizeof(float4), "prefilter row positions")))
    return -1;
  const RowRec *rowrec = shared ? (const RowRec *)c->colrec.p + roff : (const RowRec *)c->rowrec.p;
  const PFRec *pfrow = shared ? (const PFRec *)c->pfcol.p + roff : (const PFRec *)c->pfrow.p;
  const PFVel *pfvrow = shared ? (const PFVel *)c->pfvcol.p + roff : (const PFVel *)c->pfvrow.p;
  const float4 *pfprow = shared ? (const float4 *)c->pfpcol.p + roff : (const float4 *)c->pfprow.p;
  if (!shared) {  // (rows that are columns: the column word covers them)
    if (!ensure(c, c->rownf, (size_t)nrows, "row non-finite flags")) return -1;
    nfa.rowbad = (const uint8_t *)c->rownf.p;
    hipLaunchKernelGGL(k_prep_rows, dim3(blocks_for(nrows, 256)), dim3(256), 0, c->stream, (int)nrows,
                       perm_r, own, intr, rpz, hpz, tla, (RowRec *)c->rowrec.p, (PFRec *)c->pfrow.p,
                       (PFVel *)c->pfvrow.p, (float4 *)c->pfprow.p, mid, (uint8_t *)c->rownf.p, (int)rb);
    BSA_HIP(c, hipGetLastError());
  }
  // K0c for the columns is fused into K0b unless the candidate list is reused
  // (then the boxes wait for the build decision every K0b lane contributes to)
  const int nrt = (int)((nrows + kTile - 1) / kTile), nct = (int)((n + kTile - 1) / kTile);
  const long long ntp = (long long)nrt * nct;
  const int ngr = (int)((nrows + kGroup - 1) / kGroup), ngc = (int)((n + kGroup - 1) / kGroup);
  const int nsc = (int)((n + kSub - 1) / kSub);
  if (!ensure(c, c->tbox_c, nct * sizeof(TileBox), "column tile boxes") ||
      !ensure(c, c->gbox_c, ngc * sizeof(TileBox), "column group boxes") ||
      !ensure(c, c->sbox_c, nsc * sizeof(TileBox), "column sub-group boxes") ||
      !ensure(c, c->tilepairs, (size_t)ntp * kSlicesPerTile * sizeof(uint2), "prefilter items"))
    return -1;
  // tile-pair list reuse (decided above): the list's buffers and budgets
  TprArgs tp{};
  HaloTpr ht{};
  if (tpr) {
    if (!ensure(c, c->tpr_snap, (size_t)n * sizeof(PFRec), "tile-pair list snapshot")) return -1;
    const bool fresh = !c->tpr_ctl.p;
    if (!ensure(c, c->tpr_ctl, 64, "tile-pair list control")) return -1;
    if (fresh) BSA_HIP(c, hipMemsetAsync(c->tpr_ctl.p, 0, 64, c->stream));
    static const double sh_env = getenv("BSA_TPR_SH") ? atof(getenv("BSA_TPR_SH")) : 0.0;  // (A/B) [m]
    if (sh_env > 0.0) {
      c->tpr_dx = (float)(sh_env / 6.3e6);
      c->tpr_ds = (float)(sh_env / 6.3e6 / 20);
    }
    const bool force = hk ? !hkeep : !tvalid;  // (HK: the host's decision; a kept list launches no plan)
    ht = HaloTpr{halo ? 1 : 0, force ? 1 : 0, c->tpr_dx, c->tpr_ds, c->tpr_dv, (unsigned long long *)c->tpr_ctl.p,
                 nullptr};
  }
  // HK: the prediction word of this detect's records (raised by their
  // preparer -- K4' one step ago, or the own tiles' K0b here)
  unsigned long long *hk_word = hk ? (unsigned long long *)c->tpr_ctl.p + 6 + (hm & 1) : nullptr;
  FusedBoxes fb{nullptr, nullptr, nullptr, nullptr, 0};
  ZeroArgs zs{(int)nrows, 1, 0, nullptr, nullptr, nullptr, nullptr, nullptr, {}, {}};
  // halo mode: the plan's buffers are zeroed and the own tile boxes written
  // into the exchanged block by this K0b (no memset / copy launches)
  HaloPre hp{};
  if (halo && halo_pre(c, rb, re, &hp, tpr ? &ht : nullptr)) return -1;
  // plan reuse: the own K0b checks its records against the last build's and
  // raises this rank's flag (not at a forced rebuild: it rebuilds anyway)
  TprCheck tck{};
  if (tpr && halo) {
    ht.myflag = halo_flag_word(c);
    if (!ht.force)
      tck = TprCheck{(const PFRec *)c->tpr_snap.p, ht.myflag, c->tpr_dx, c->tpr_ds, c->tpr_dv, hk_word, c->hk_f};
  }
  if (!reuse) {
    fb = FusedBoxes{(TileBox *)c->sbox_c.p, (TileBox *)c->gbox_c.p, (TileBox *)c->tbox_c.p, hp.blk, hp.blk_base};
    zs = ZeroArgs{(int)nrows, 1, 0, dcnt, (unsigned long long *)c->workq.p, (unsigned char *)c->inconf.p,
                  (unsigned long long *)c->tcpamax.p, (unsigned *)c->rowcnt.p, {hp.z[0], hp.z[1], hp.z[2]},
                  {hp.zn[0], hp.zn[1], hp.zn[2]}};
  }
  const int na = halo ? a1 - a0 : 0;
  // halo overlap (Ctx::ov_mode): a kept plan of several ranks (mode 2: also the
  // probe) sweeps the own column tiles on the stream while the exchange, the
  // received tiles' K0b and their sweep run on xstream
  const bool ovl = halo && hkeep && !noprune && na > 0 && (c->ov_mode == 2 || (c->ov_mode == 1 && c->halo_mode == 1));
  if (ovl && ov_init(c)) return -1;
  if (prepped) {  // K0b + K0c ran in the previous step's K4': K0z + the tile boxes here
    if (!nozero && zero(false, nullptr, 0, true)) return -1;
  } else if (!(halo && hkeep)) {  // (HK keep, several ranks: the own tiles go with the halo tiles below)
    const unsigned g = halo ? (unsigned)na : blocks_for(n, kTile);
    hipLaunchKernelGGL(k_prep_cols, dim3(g), dim3(kTile), 0, c->stream, (int)n, perm_c, home ? 1 : 0,
                       recs ? 1 : 0, own, intr, distinct ? 1 : 0, shared ? 1 : 0, rpz, hpz, tla,
                       (ColRec *)c->colrec.p, (PFRec *)c->pfcol.p, (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, mid,
                       rz, fb, zs, halo ? a0 : 0, (const int *)nullptr, HaloUnpack{}, (Counters *)nullptr, tck, nfa,
                       (int)g);
  }
  BSA_HIP(c, hipGetLastError());
  if (halo) {
    HaloUnpack hu{};
    // (halo overlap: K0z before the pack -- xstream's K0b writes Counters)
    if (ovl && !nozero && zero(false, nullptr, 0)) return -1;
    if (halo_mid(c, rb, re, &hu, tpr ? &ht : nullptr, hkeep, ovl && c->halo_mode == 1 ? c->xstream : nullptr))
      return -1;
    const ZeroArgs zs2{(int)nrows, 1, 0, nullptr, nullptr, nullptr, nullptr, nullptr, {}, {}};
    FusedBoxes fb2 = fb;
    fb2.blk = nullptr;
    hu.count = halo_list_count(c);
    if (ovl) {
      // the own tiles (budget checks included) on the stream; the received
      // ones on xstream once the exchange is in (the probe: no exchange, after
      // K0z), which then waits for the own tiles (its sweep's rows)
      if (c->halo_mode != 1) {
        BSA_HIP(c, hipEventRecord(c->ov_ev[0], c->stream));
        BSA_HIP(c, hipStreamWaitEvent(c->xstream, c->ov_ev[0], 0));
      }
      hipLaunchKernelGGL(k_prep_cols, dim3((unsigned)na), dim3(kTile), 0, c->stream, (int)n, perm_c, 1, recs ? 1 : 0,
                         own, intr, 0, 1, rpz, hpz, tla, (ColRec *)c->colrec.p, (PFRec *)c->pfcol.p,
                         (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, mid, rz, fb2, zs2, a0, (const int *)nullptr,
                         HaloUnpack{}, (Counters *)nullptr, tck, nfa, na);
      BSA_HIP(c, hipGetLastError());
      BSA_HIP(c, hipEventRecord(c->ov_ev[1], c->stream));
      if (c->halo_hl > 0) {
        hipLaunchKernelGGL(k_prep_cols, dim3((unsigned)c->halo_hl), dim3(kTile), 0, c->xstream, (int)n, perm_c, 1,
                           recs ? 1 : 0, own, intr, 0, 1, rpz, hpz, tla, (ColRec *)c->colrec.p,
                           (PFRec *)c->pfcol.p, (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, mid, rz, fb2, zs2, 0,
                           (const int *)c->h_hl.p, hu, dcnt, TprCheck{}, nfa, 0);
        BSA_HIP(c, hipGetLastError());
      }
      BSA_HIP(c, hipStreamWaitEvent(c->xstream, c->ov_ev[1], 0));
    } else if (hkeep) {
      // HK keep: no plan, so the own tiles wait for nothing before the
      // exchange -- ONE K0b for them and the received tiles (workgroups [0, na)
      // the own tiles with their budget checks, the rest the halo list's
      // slots); K0z is K2's (double-buffered counters) or its own launch,
      // never inside it (its halo workgroups write Counters)
      if (!nozero && zero(false, nullptr, 0)) return -1;
      hipLaunchKernelGGL(k_prep_cols, dim3((unsigned)(na + c->halo_hl)), dim3(kTile), 0, c->stream, (int)n, perm_c,
                         1, recs ? 1 : 0, own, intr, 0, 1, rpz, hpz, tla, (ColRec *)c->colrec.p,
                         (PFRec *)c->pfcol.p, (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, mid, rz, fb2, zs2, a0,
                         (const int *)c->h_hl.p, hu, dcnt, tck, nfa, na);
      BSA_HIP(c, hipGetLastError());
    } else if (c->halo_hl > 0) {  // the received tiles: unpacked (exchange), records and boxes (no zeroing here)
      hipLaunchKernelGGL(k_prep_cols, dim3((unsigned)c->halo_hl), dim3(kTile), 0, c->stream, (int)n, perm_c, 1,
                         recs ? 1 : 0, own, intr, 0, 1, rpz, hpz, tla, (ColRec *)c->colrec.p,
                         (PFRec *)c->pfcol.p, (PFVel *)c->pfvcol.p, (float4 *)c->pfpcol.p, mid, rz, fb2, zs2, 0,
                         (const int *)c->h_hl.p, hu, dcnt, TprCheck{}, nfa, 0);
      BSA_HIP(c, hipGetLastError());
    }
  }

  // ---- K0c/K0d group / tile boxes (rows; columns when reused) and the tile-pair work list
  if (!shared && (!ensure(c, c->tbox_r, nrt * sizeof(TileBox), "row tile boxes") ||
                  !ensure(c, c->gbox_r, ngr * sizeof(TileBox), "row group boxes")))
    return -1;
  const TileBox *gbox_r = shared ? (const TileBox *)c->gbox_c.p + roff / kGroup : (const TileBox *)c->gbox_r.p;
  const TileBox *tbox_r = shared ? (const TileBox *)c->tbox_c.p + roff / kTile : (const TileBox *)c->tbox_r.p;
  if (!shared)
    hipLaunchKernelGGL(k_boxes, dim3(nrt), dim3(kTile), 0, c->stream, (int)nrows, pfrow, (TileBox *)nullptr,
                       (TileBox *)c->gbox_r.p, (TileBox *)c->tbox_r.p, build, (Counters *)nullptr);
  if (reuse)
    hipLaunchKernelGGL(k_boxes, dim3(nct), dim3(kTile), 0, c->stream, (int)n, (const PFRec *)c->pfcol.p,
                       (TileBox *)c->sbox_c.p, (TileBox *)c->gbox_c.p, (TileBox *)c->tbox_c.p, build, dcnt);
  // ~1024 workgroups' worth of candidates per thread-chunk (one at 100k, several at 1M)
  const unsigned long long icap = (unsigned long long)ntp * kSlicesPerTile;  // items: 8 slices per tile pair
  if (tpr)  // (after halo_mid, which may have forced the rebuild)
    tp = TprArgs{(unsigned long long *)c->tpr_ctl.p, ht.force, c->tpr_dx, c->tpr_ds, c->tpr_dv,
                 (const PFRec *)c->pfcol.p + roff, (PFRec *)c->tpr_snap.p + roff, halo ? ht.myflag : nullptr,
                 hkeep ? 1 : 0, hkeep ? (halo ? ht.myflag : (const unsigned *)c->tpr_ctl.p) : nullptr,
                 hkeep && c->sim_ctl.p ? (unsigned long long *)((char *)c->sim_ctl.p + kSimCtlStale) : nullptr};
  if (hkeep) {
    // HK keep: no K0d -- the prefilter takes the kept list's counts from the control words
  } else if ((nct <= kTPDirectMax || tp_list) && !tp_super)
    hipLaunchKernelGGL(k_tilepairs_direct, dim3((unsigned)nrt), dim3(kTPDirectThreads), 0, c->stream, nrt, nct,
                       (int)nrows, tbox_r, gbox_r, (const TileBox *)c->tbox_c.p, noprune, (uint2 *)c->tilepairs.p,
                       icap, dcnt, (unsigned long long *)c->workq.p, build, halo ? halo_present(c) : nullptr, a0,
                       a1, nozero ? (const TileBox *)c->gbox_c.p : (const TileBox *)nullptr,
                       tp_list ? (const int *)c->h_hl.p : (const int *)nullptr, (int)c->halo_hl,
                       tp_list ? halo_list_count(c) : (const unsigned *)nullptr, tp);
  else
    hipLaunchKernelGGL(k_tilepairs, dim3((unsigned)((nrt + kSuper - 1) / kSuper)), dim3(kTPThreads), 0, c->stream,
                       nrt, nct, (int)nrows, tbox_r, gbox_r, (const TileBox *)c->tbox_c.p, noprune,
                       (uint2 *)c->tilepairs.p, icap, dcnt, (unsigned long long *)c->workq.p, build,
                       halo ? halo_present(c) : nullptr, a0, a1);
  BSA_HIP(c, hipGetLastError());
  if (mark(1)) return -1;

  const float T = (float)(tla > 0.0 ? tla : 0.0);
  const float lim = (float)((rpz + kEABS + (reuse ? 2.0 * c->reuse_sh : 0.0)) / (1.0 - kE1));
  const float liml = lim / kRS;  // unit-sphere units (pf_refine)
  const RefineParams rp{(float)rpz, (float)hpz, T, kwik ? INFINITY : liml * liml, 0.f};
  // ---- K1a prefilter: persistent grid, PF_BLOCKS_PER_CU workgroups per CU
  // (LDS-limited residency), at least one workgroup per dequeue shard
  // pieces: ~8 items per row tile, a few hundred row tiles fill the waves;
  // fewer rows split the items (BSA_PF_PIECES overrides)
  static const int pieces_env = getenv("BSA_PF_PIECES") ? atoi(getenv("BSA_PF_PIECES")) : 0;
  PfKnobs kn{1, 1, 1, 0, 0, 0};
  static const int t0_env = getenv("BSA_PF_HEAVY_T0") ? atoi(getenv("BSA_PF_HEAVY_T0")) : -1;
  if (t0_env >= 0 && t0_env <= 3) kn.t0 = t0_env;
  // (measured, tools/gpu_pieces.sh: 2 pieces at the 100k box, 102 -> 97 us; 4 for
  // one rank of 8 there, 36 -> 29 us; 2 at 125k rows of 1M, 65 -> 53 us; 1
  // from 250k rows up, where 2 cost +15 us.  Round 5, with the longest-items
  // listing and the fused K1b: 1 piece from 64k rows up -- the 100k box
  // 0.1204 / 0.1212 -> 0.1185 / 0.1181 ms per step, one rank of 8 at 1M
  // 0.1130 / 0.1117 -> 0.1118 / 0.1112; tools/gpu_ab.sh, BSA_PF_PIECES=1),
  // 2 from 16k rows: one rank of 4 at the 100k box (25k rows) 0.0942 / 0.0938
  // -> 0.0925 / 0.0912 (tools/probe_step.py), of 8 (12.8k rows) stays at 4
  kn.pieces = nrows >= (1 << 16) ? 1 : (nrows >= (1 << 14) ? 2 : 4);
  if (pieces_env == 1 || pieces_env == 2 || pieces_env == 4 || pieces_env == 8) kn.pieces = pieces_env;
  static const int pnear_env = getenv("BSA_PF_PIECES_NEAR") ? atoi(getenv("BSA_PF_PIECES_NEAR")) : 0;
  kn.pnear = kn.pieces;
  if (pnear_env == 1 || pnear_env == 2 || pnear_env == 4 || pnear_env == 8) kn.pnear = pnear_env;
#ifdef BSA_PF_TRACE
  {
    static DevBuf tb;
    const size_t need = (size_t)kTraceRecs * 32;
    if (!ensure(c, tb, need, "prefilter trace")) return -1;
    BSA_HIP(c, hipMemsetAsync(tb.p, 0, need, c->stream));
    void *pt = tb.p;
    BSA_HIP(c, hipMemcpyToSymbolAsync(HIP_SYMBOL(pf_trace), &pt, sizeof pt, 0, hipMemcpyHostToDevice, c->stream));
    c->trace_buf = tb.p;
    c->trace_bytes = need;
  }
#endif
  // longest items first (HeavyArgs): detects of a kept tile-pair list only
  // (Ctx::hv_us: the listing threshold, < 0 off)
  HeavyArgs hv{};
  HeavyNext hn{};
  if (tpr && c->hv_us >= 0.0) {
    const bool fresh = c->hv_icap != icap || !c->hv_cnt.p;
    if (!ensure(c, c->hv_cost, icap * 4, "item costs") || !ensure(c, c->hv_flag, icap * 4, "listed item flags") ||
        !ensure(c, c->hv_list[0], icap * 4, "listed items") || !ensure(c, c->hv_list[1], icap * 4, "listed items") ||
        !ensure(c, c->hv_list[2], icap * 4, "listed items") || !ensure(c, c->hv_list[3], icap * 4, "listed items") ||
        !ensure(c, c->hv_cnt, 64, "listed item counts"))
      return -1;
    if (fresh) {
      BSA_HIP(c, hipMemsetAsync(c->hv_cost.p, 0, icap * 4, c->stream));
      BSA_HIP(c, hipMemsetAsync(c->hv_flag.p, 0, icap * 4, c->stream));
      BSA_HIP(c, hipMemsetAsync(c->hv_cnt.p, 0, 64, c->stream));
      c->hv_icap = icap;
    }
    const unsigned E = ++c->hv_epoch;  // (flags hold epochs >= 1; 0 = never)
    unsigned *cn = (unsigned *)c->hv_cnt.p;
    const unsigned a = E & 1, b = (E + 1) & 1;  // this detect's / the next one's lists and counts
    const double x = c->hv_x > 0.0 ? c->hv_x : 1e30;  // (tier 0 off: no slot reaches it)
    // a rank's share (halo mode) sweeps in ~40 us, not ~70: half the threshold
    // (one rank of 8 at global1m, probe A/B x 3: 0.1010-0.1029 -> 0.1007-0.1009
    // ms per step at 8 us, 0.0995-0.1010 at 5; box100k unchanged at 16)
    const double us = halo && !c->hv_us_env ? 0.5 * c->hv_us : c->hv_us;
    hv = HeavyArgs{{(const unsigned *)c->hv_list[2 * a].p, (const unsigned *)c->hv_list[2 * a + 1].p}, cn + 2 * a,
                   cn + 2 * b, (const unsigned *)c->hv_flag.p, (unsigned *)c->hv_cost.p, E};
    hn = HeavyNext{(unsigned *)c->hv_cost.p, {(unsigned *)c->hv_list[2 * b].p, (unsigned *)c->hv_list[2 * b + 1].p},
                   cn + 2 * b, (unsigned *)c->hv_flag.p, E + 1,
                   {(unsigned)std::min(us * x * 100.0, 4e9), (unsigned)std::min(us * 100.0, 4e9)},
                   // the list's item counts: ctl[1], ctl[2] (the prefilter publishes a built list's there;
                   // an HK-kept detect fills no dequeue words)
                   (const unsigned long long *)c->tpr_ctl.p, icap};
  }
  // K2 row buckets (B pairs per row per list; a fuller row retries wider, then without)
  const int B = c->k2_bucket;
  if (B && !ensure(c, c->kbuck, (size_t)2 * nrows * B * sizeof(uint2), "K2 row buckets")) return -1;
  // K1b fused into the prefilter (ExactFuse): stored records, row buckets, no
  // KWIK / candidate reuse, not one rank's share of a sharded step (there the
  // sweep is short and the workgroups' end-of-sweep evaluation lengthened it
  // more than K1b's launch cost: global1m rank 2 of 8, prefilter 46 + K1b 11
  // -> 63 us; box100k one rank: 0.1387-0.1396 -> 0.1336-0.1367 ms per step).
  // BSA_FUSE_EXACT=0/1 overrides (A/B).
  static const int fuse_env = getenv("BSA_FUSE_EXACT") ? atoi(getenv("BSA_FUSE_EXACT")) : -1;
  const bool fuse = fuse_env != 0 && (fuse_env == 1 || !halo) && c->fuse_on && !c->fuse_skip && B > 0 && recs &&
                    !kwik && !reuse && !ovl;
  c->fuse_skip = false;  // (one retry unfused; the next detect fuses again)
  ExactFuse xf{};
  if (fuse)
    xf = ExactFuse{rowrec, (const ColRec *)c->colrec.p, perm_r, perm_c, rpz, hpz, tla, (int)rb, (int)nrows, B,
                   (double *)c->cpay.p, (unsigned *)c->rowcnt.p, (uint2 *)c->kbuck.p, (unsigned)c->fuse_recs};
  c->last_fused = fuse;
  if (fuse) c->fuse_count++;
  // rows sharing the column records: row i is column roff + i (its diagonal)
  const int diag = shared ? (int)roff : -1;
  const unsigned pf_grid = (unsigned)std::max<long long>(
      kWorkShards, std::min<long long>(ntp * PF_ITEMS_PER_TILE / PF_WAVES + 1, 256 * PF_BLOCKS_PER_CU));
  if (noprune)
    hipLaunchKernelGGL(k_prefilter<true>, dim3(pf_grid), dim3(PF_BLOCK), 0, c->stream, pfrow, pfvrow, pfprow,
                       (int)nrows, (const PFRec *)c->pfcol.p, (const PFVel *)c->pfvcol.p,
                       (const float4 *)c->pfpcol.p, (int)n, gbox_r, (const TileBox *)c->sbox_c.p, noprune,
                       (const uint2 *)c->tilepairs.p, icap, dcnt,
                       (unsigned long long *)c->workq.p, rp, (uint2 *)c->cand.p, cap, build, kn, diag, TprArgs{},
                       HeavyArgs{}, xf);
  else
    for (int ph = ovl ? 1 : 0; ph <= (ovl ? 2 : 0); ++ph) {  // (halo overlap: own tiles here, the others on xstream)
      PfKnobs kp = kn;
      kp.ph = ph;
      kp.ca0 = a0;
      kp.ca1 = a1;
      // (the own tiles' sweep leaves half the workgroup slots to the received
      // tiles' K0b and sweep: 2 of 4 per CU, BSA_OV_GRID_A; probe with the
      // overlap 0.134 ms per step at 4, 0.121 at 2, 0.104 without it)
      static const int ga = getenv("BSA_OV_GRID_A") ? atoi(getenv("BSA_OV_GRID_A")) : 2;
      const unsigned g = ph == 1 && ga > 0 ? std::min<unsigned>(pf_grid, std::max(256u * (unsigned)ga, (unsigned)kWorkShards)) : pf_grid;
      hipLaunchKernelGGL(k_prefilter<false>, dim3(g), dim3(PF_BLOCK), 0, ph == 2 ? c->xstream : c->stream,
                         pfrow, pfvrow, pfprow, (int)nrows, (const PFRec *)c->pfcol.p, (const PFVel *)c->pfvcol.p,
                         (const float4 *)c->pfpcol.p, (int)n, gbox_r, (const TileBox *)c->sbox_c.p, noprune,
                         (const uint2 *)c->tilepairs.p, icap, dcnt,
                         (unsigned long long *)c->workq.p, rp, (uint2 *)c->cand.p, cap, build, kp, diag, tp, hv, xf);
      BSA_HIP(c, hipGetLastError());
    }
  if (ovl) {  // join: K1b on waits for the halo tiles' sweep
    BSA_HIP(c, hipEventRecord(c->ov_ev[2], c->xstream));
    BSA_HIP(c, hipStreamWaitEvent(c->stream, c->ov_ev[2], 0));
    c->ov_count++;
  }
  BSA_HIP(c, hipGetLastError());
  if (mark(2)) return -1;
  // ---- K1b exact evaluation: grid-stride over the device-side count of the
  // dense candidate list; 2048 workgroups (524 k lanes: the 100k box's ~153 k
  // candidates in one stride, the workgroups past the count exit at once;
  // BSA_K1B_GRID overrides for A/B)
  if (!fuse) {
    const auto KEX = !recs ? k_exact<kExactHome> : (kwik ? k_exact<kExactKwik> : k_exact<kExactRec>);
    static const int k1b_grid = getenv("BSA_K1B_GRID") ? atoi(getenv("BSA_K1B_GRID")) : 0;
    hipLaunchKernelGGL(KEX, dim3(k1b_grid > 0 ? (unsigned)k1b_grid : 256u * 8u), dim3(256), 0, c->stream, rowrec, (const ColRec *)c->colrec.p,
                       perm_r, perm_c, (const uint2 *)c->cand.p, dcnt, own, cap, rpz, hpz, tla, (int)rb,
                       (int)nrows,
                       (unsigned char *)c->cflag.p, (double *)c->cpay.p,
                       (unsigned char *)c->inconf.p, (unsigned long long *)c->tcpamax.p,
                       (unsigned *)c->rowcnt.p, (uint2 *)c->kbuck.p, B,
                       reuse ? (unsigned *)c->reuse_ctl.p : nullptr,
                       (const Snap *)c->snap_cur.p, (Snap *)c->snap_build.p, (int)n, hn);
  }
  BSA_HIP(c, hipGetLastError());
  if (mark(3)) return -1;
  // ---- K2: row offsets and the pairs in row-major order: from K1b's row
  // buckets (k_rank_rows, one launch), or scan + scatter into row segments +
  // per-segment rank (bucket width 0)
  if (!B) {
    const int nscan = (int)(2 * (nrows + 1));
    if (scan_excl(c, (const unsigned *)c->rowcnt.p, (unsigned *)c->rowoff.p, nscan)) return -1;
    hipLaunchKernelGGL(k_scatter, dim3(256 * 4), dim3(256), 0, c->stream, (const Counters *)dcnt, cap, (int)rb,
                       (int)nrows, (const unsigned char *)c->cflag.p, (const double *)c->cpay.p,
                       (const unsigned *)c->rowoff.p, (unsigned *)c->rowcnt.p,
                       (unsigned long long *)c->ckey2.p, (unsigned *)c->cval2.p,
                       (unsigned long long *)c->lkey2.p);
    BSA_HIP(c, hipGetLastError());
  }
  MvpFuse mf{};
  c->fuse_done = false;
  c->fuse_rowdv = false;
  if (c->fuse_mvp) {
    if (!ensure(c, c->mvp_pdv, std::max<unsigned long long>(cap, 1) * sizeof(double4), "mvp pair dv") ||
        !ensure(c, c->mvp_pfl, std::max<unsigned long long>(cap, 1), "mvp pair flags"))
      return -1;
    mf.p = *c->fuse_mvp;
    mf.in = MvpPairIn{c->fuse_gse, c->fuse_gsn, c->fuse_vs, c->fuse_alt, c->fuse_noreso,
                      c->det_home ? (const unsigned *)c->id2h.p : nullptr};
    mf.pdv = (double4 *)c->mvp_pdv.p;
    mf.pfl = (uint8_t *)c->mvp_pfl.p;
    c->fuse_done = true;
    if (B) {  // K2 also folds each row's vectors (MvpIn::rowdv)
      if (!ensure(c, c->mvp_rowdv, (size_t)std::max<int64_t>(nrows, 1) * sizeof(double4), "mvp row dv")) return -1;
      mf.rowdv = (double4 *)c->mvp_rowdv.p;
      c->fuse_rowdv = true;
    }
  }
  if (B) {
    const bool hl = fuse && hn.cost;  // the heavy-item listing moves here from K1b
    hipLaunchKernelGGL(k_rowblk, dim3((unsigned)((rank_blocks((int)nrows) + kRowblkWaves - 1) / kRowblkWaves) +
                                          (hl ? kHeavyBlocks : 0u)),
                       dim3(64 * kRowblkWaves), 0,
                       c->stream, (int)nrows, (unsigned *)c->rowcnt.p, hl ? hn : HeavyNext{});
    const RankLaunch rl{(unsigned)rank_blocks((int)nrows), (int)nrows, dcnt, cap, (unsigned *)c->rowoff.p,
                        (unsigned *)c->rowcnt.p, (const uint2 *)c->kbuck.p, B, (const double *)c->cpay.p, (int)rb,
                        (int *)c->out_ci.p, (int *)c->out_cj.p, (double *)c->out_pay.p, (int *)c->out_li.p,
                        (int *)c->out_lj.p, (unsigned long long *)c->stats.p, gate, build, mf,
                        (unsigned char *)c->inconf.p, (unsigned long long *)c->tcpamax.p,
                        (Counters *)c->counters2.p, (unsigned long long *)c->workq2.p, nfa, hk_word};
    if (c->k24_want) {  // bsa_sim_step launches it fused with K4' (k24_launch)
      c->k24_blob.resize(sizeof rl);
      memcpy(c->k24_blob.data(), &rl, sizeof rl);
      c->k24_pending = true;
      c->k24_ev = timed ? ev[4] : nullptr;
    } else {
      rank_launch(c, rl, false, K24Args{});
    }
    c->zeroed_rows = nrows;
  } else {
    hipLaunchKernelGGL(k_rank, dim3(256 * 4), dim3(256), 0, c->stream, (int)nrows, dcnt, cap,
                       (const unsigned *)c->rowoff.p, (const unsigned long long *)c->ckey2.p,
                       (const unsigned *)c->cval2.p, (const double *)c->cpay.p,
                       (const unsigned long long *)c->lkey2.p, (int)rb, (int *)c->out_ci.p, (int *)c->out_cj.p,
                       (double *)c->out_pay.p, (int *)c->out_li.p, (int *)c->out_lj.p,
                       (unsigned long long *)c->stats.p, gate, build, mf, nfa, (unsigned long long *)c->tcpamax.p);
  }
  BSA_HIP(c, hipGetLastError());
  if (!c->k24_pending && mark(4)) return -1;
  c->ev_valid = c->ev_valid || timed;
  return 0;
}

// the K2 launch kept by detect_enqueue, fused with the step's K4'
int k24_launch(Ctx *c, const K24Args &ka) {
  if (!c->k24_pending || c->k24_blob.size() != sizeof(RankLaunch)) return fail(c, "internal: no K2 launch to fuse");
  RankLaunch rl;
  memcpy(&rl, c->k24_blob.data(), sizeof rl);
  c->k24_pending = false;
  if (rank_launch(c, rl, true, ka)) return -1;
  if (c->k24_ev) BSA_HIP(c, hipEventRecord(c->k24_ev, c->stream));
  c->k24_ev = nullptr;
  return 0;
}

// K2 row buckets too narrow for a row with `demand` pairs: the next power of
// two, or (beyond 64) the scatter into row segments
void grow_k2_bucket(Ctx *c, unsigned long long demand) {
  int b = std::max(c->k2_bucket, 1);
  while ((unsigned long long)b < demand && b <= 64) b *= 2;
  c->k2_bucket = b > 64 ? 0 : b;
}

#ifdef BSA_PF_TRACE
// diagnostic builds: the last prefilter's item timeline to $BSA_PF_TRACE_FILE
// (tools/pf_trace.py; detect_finish, and bsa_sim_step after each batch)
int pf_trace_dump(Ctx *c, unsigned long long groups, unsigned long long tiles) {
  const char *fn = getenv("BSA_PF_TRACE_FILE");
  if (!fn || !c->trace_buf) return 0;
  std::vector<unsigned long long> t(kTraceRecs * 4);
  BSA_HIP(c, hipMemcpy(t.data(), c->trace_buf, t.size() * 8, hipMemcpyDeviceToHost));
  if (FILE *f = fopen(fn, "ab")) {
    const unsigned long long hdr[4] = {0xfeedull, (unsigned long long)(t.size() / 4), groups, tiles};
    fwrite(hdr, 8, 4, f);
    fwrite(t.data(), 8, t.size(), f);
    fclose(f);
  }
  return 0;
}
#endif

// Wait for the enqueued detect and read its totals.  *retry is set (and the
// candidate capacity grown) when the candidate list overflowed.
int detect_finish(Ctx *c, bool *retry) {
  *retry = false;
  Counters h;
  BSA_HIP(c, hipMemcpyAsync(&h, c->counters.p, sizeof(Counters), hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  if (c->empty_detect) {
    c->last_conf = c->last_los = c->last_cand = c->last_tiles = c->last_groups = 0;
    c->have_pairs = true;
    return 0;
  }
  c->zeroed_rows = -1;  // (a retry zeroes everything again; so does any host-side recovery)
  // every cause of a retry is fixed before the one retry (not one per retry)
  if (h.fuse_ovf) {  // a wave flushed more blocks than the fused K1b records: K1b as its own launch
    c->fuse_skip = true;
    c->fuse_retries++;
    *retry = true;
  }
  if (h.k2_demand) {  // a K2 row bucket was full: nothing was written (the
    grow_k2_bucket(c, h.k2_demand);  // candidate list itself is complete: a reusable one stays valid)
    *retry = true;
  }
  unsigned long long worst = 0;
  for (int q = 0; q < kCandShards; ++q) worst = std::max(worst, h.cshard[q][0]);
  const unsigned long long total = h.cand;  // (the list is dense: K2 summed the shard counts)
  if (worst > c->cand_cap / kCandShards) {
    c->cand_cap = (unsigned long long)kCandShards * (worst + worst / 4 + 1024);
    c->reuse_valid = false;
    *retry = true;
  }
  if (*retry) return 0;
  const int64_t nrows = c->last_re - c->last_rb;
  c->last_cand = (int64_t)total;
  c->last_tiles = (int64_t)h.tiles;
  c->last_tiles_total = (int64_t)(((nrows + kTile - 1) / kTile) * ((c->n + kTile - 1) / kTile));
  c->last_groups = (int64_t)h.groups;
  c->last_conf = (int64_t)h.conf;
  c->last_los = (int64_t)h.los;
  c->have_pairs = true;
#ifdef BSA_PF_TRACE
  if (pf_trace_dump(c, h.groups, h.tiles)) return -1;
#endif
#ifdef BSA_PF_STAMPS
  fprintf(stderr, "[bsa stamps] prefilter wave-cycles: setup %.4g stage1 %.4g drain %.4g flush %.4g | "
          "stage-1 survivors %.4g refine rounds %.4g batches %.4g enqueue trips %.4g\n",
          (double)h.stamp[0], (double)h.stamp[1], (double)h.stamp[2], (double)h.stamp[3], (double)h.stamp[4],
          (double)h.stamp[5], (double)h.stamp[6], (double)h.stamp[7]);
#endif
  return 0;
}

int detect(Ctx *c, double rpz, double hpz, double tla, int flags, int64_t rb, int64_t re,
           int64_t *n_conf, int64_t *n_los) {
  for (int attempt = 0;; ++attempt) {
    if (detect_enqueue(c, rpz, hpz, tla, flags, rb, re, nullptr)) return -1;
    bool retry = false;
    if (detect_finish(c, &retry)) return -1;
    if (!retry) break;
    if (attempt >= 4) return fail(c, "candidate buffer overflow after %d retries", attempt + 1);
  }
  *n_conf = c->last_conf;
  *n_los = c->last_los;
  return 0;
}

}  // namespace bsa
