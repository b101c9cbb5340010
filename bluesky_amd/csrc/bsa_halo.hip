// Halo exchange of the row-sharded resident step.
//
// Rank r owns the home rows [r rpr, (r + 1) rpr): a spatially compact chunk
// of the traffic whose 512-row tiles are column tiles of the detect.  Its
// rows can only conflict with column tiles whose boxes pass the tile-pair
// test (boxes_may_interact, bsa_box.h) against one of its row tiles, so
// instead of all-gathering the whole state before every CD call (48 MB at 1M
// aircraft) each rank
//   1. prepares its OWN column tiles (K0b, with their boxes), which also
//      zeroes the plan's buffers and writes its tile boxes into the block it
//      sends (no memset / copy launches: every launch boundary costs ~4.5 us);
//   2. all-gathers the tile boxes (48 B per tile) and a request bitmask of the
//      tiles holding its resopairs' intruders (ResumeNav reads their state,
//      asas.py:424-452, wherever they are by now);
//   3. plans (k_halo_plan + k_halo_lists): tile t of rank s goes to rank q iff
//      t passes the box test against some row tile of q, or q requested it --
//      every rank evaluates the same test on the same (gathered, bitwise) boxes
//      from its own side, and the test is symmetric, so sender and receiver
//      agree;
//   4. exchanges the planned tiles' state (lat lon trk gs alt vs, and gseast /
//      gsnorth unless they follow from gs / trk) with one grouped RCCL
//      send / recv per neighbour (device copies in the in-process group),
//      into the same home positions of the replicated arrays;
//   5. unpacks and prepares the received tiles (one K0b over the flat halo
//      list: each workgroup unpacks its tile's rows, then prepares them).
// K0d (k_tilepairs) then lists tile pairs of present column tiles only; a
// kept pair with a missing tile would be a plan bug and is flagged
// (Counters::halo_miss: the step fails loudly), never swept with stale data.
// K1b, MVP's per-pair vectors and the bookkeeping read rows of present tiles
// only.
//
// RCCL takes host-side sizes, so every (sender, receiver) pair has a tile
// capacity, the same on all ranks: exact at bsa_sim_init (every rank holds the
// whole initial state and plans for all ranks), grown when a step needs more
// (Counters::halo_ovf aborts the step like a candidate overflow, the demands
// are max-all-reduced on the host, every rank grows the same capacities and
// the step re-runs).  A capacity's region is always sent whole: a count and
// the tile ids, then the tiles' rows.
//
// The one-GPU probe of one rank's share (bsa_sim_detect_rows, mode 2) runs
// steps 1, 3 and 5 with every tile's box already on the GPU.
#include <algorithm>

#include "bsa_box.h"
#include "bsa_halo.h"
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

static inline size_t region_bytes(int cap, int nf) {
  return cap ? halo_hdr_bytes(cap) + (size_t)cap * halo_tile_bytes(nf) : 0;
}

// requests: the tiles of this rank's resopairs' intruders outside its own tiles
// (with plan reuse: a requested tile this rank does not hold -- present, the
// kept plan's mask -- raises its rebuild flag, so the next plan delivers it)
__global__ __launch_bounds__(256) void k_halo_req(int nrows, const unsigned *__restrict__ rptr,
                                                  const unsigned *__restrict__ rcol, const unsigned *__restrict__ id2h,
                                                  int a0, int a1, unsigned *__restrict__ req,
                                                  const uint8_t *__restrict__ present, unsigned *__restrict__ flag) {
  const unsigned total = rptr[nrows];
  for (unsigned k = blockIdx.x * blockDim.x + threadIdx.x; k < total; k += gridDim.x * blockDim.x) {
    const unsigned j = rcol[k];
    if (j == kDangling) continue;
    const int t = (int)(id2h[j] / (unsigned)kTile);
    if (t < a0 || t >= a1) {
      atomicOr(&req[t >> 5], 1u << (t & 31));
      if (flag && !present[t]) *flag = 1u;
    }
  }
}

struct PlanArgs {
  int nct, tpr, R, me, a0, a1;
  const TileBox *tbox;        // own tile boxes (probe: every tile's)
  const unsigned char *gblk;  // gathered blocks [R][tpr boxes | request words | flag word], or NULL (probe)
  size_t bb;                  // block bytes
  TileBox *tbox_out;          // exchange: the gathered boxes of other ranks' tiles -> tbox_c
  uint8_t *recv;              // [nct] tiles this rank needs (the present mask besides its own)
  uint8_t *send;              // [R][tpr] own tiles each rank needs (exchange), else NULL
  int W;                      // request words per block
  HaloTpr ht;                 // plan reuse (ht.tpr = 0: plan every detect)
  unsigned *dem;              // demand words (zeroed here at a rebuild with reuse), 2 Rd + 1
  int ndem;
};

__device__ __forceinline__ const TileBox &plan_box(const PlanArgs &a, int t) {
  if (!a.gblk) return a.tbox[t];
  const int q = t / a.tpr;
  return reinterpret_cast<const TileBox *>(a.gblk + (size_t)q * a.bb)[t - q * a.tpr];
}
__device__ __forceinline__ bool req_bit(const PlanArgs &a, int q, int t) {
  const unsigned *w = reinterpret_cast<const unsigned *>(a.gblk + (size_t)q * a.bb + (size_t)a.tpr * sizeof(TileBox));
  return (w[t >> 5] >> (t & 31)) & 1u;
}

// ordered compaction of flag(0 .. m-1) by one 256-lane workgroup: f(index,
// rank) for every set flag; returns the count (every lane)
template <typename Flag, typename F>
__device__ __forceinline__ int block_compact(int m, Flag flag, F f) {
  __shared__ int wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int base = 0;
  for (int c0 = 0; c0 < m; c0 += 256) {
    const int i = c0 + (int)threadIdx.x;
    const bool on = i < m && flag(i);
    const unsigned long long b = __ballot(on);
    const int before = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(b);
    __syncthreads();
    int off = base;
    for (int q = 0; q < w; ++q) off += wsum[q];
    if (on) f(i, off + before);
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  return base;
}

struct ListArgs {
  int nct, tpr, R, me, a0, a1;
  int probe;                     // one-GPU probe: source q's slots are [q tpr, (q + 1) tpr), no sends
  const uint8_t *recv, *send;
  int *hl;                       // flat halo list (this rank's receive slots)
  unsigned char *sbuf;           // h_send (the region headers are written here)
  unsigned *dem;                 // [R] send demand, [R] receive demand, [2R] tiles received
  Counters *cnt;
};

// the ordered list of own tiles rank q needs (into the header of the send
// region for q) and of rank q's tiles this rank needs (into the flat list)
__device__ void halo_lists_q(const ListArgs &a, const HaloCaps &cp, int q) {
  if (q == a.me) return;
  const int na = a.a1 - a.a0;
  bool ovf = false;
  if (!a.probe) {
    unsigned *hdr = reinterpret_cast<unsigned *>(a.sbuf + cp.soff[q]);
    const int cap = cp.scap[q];
    const int sc = block_compact(na, [&](int i) { return a.send[(size_t)q * a.tpr + i] != 0; },
                                 [&](int i, int k) { if (k < cap) hdr[1 + k] = (unsigned)(a.a0 + i); });
    if (threadIdx.x == 0) {
      if (cap) hdr[0] = (unsigned)min(sc, cap);
      a.dem[q] = (unsigned)sc;
    }
    ovf = sc > cap;
  }
  const int t0 = q * a.tpr, t1 = min(a.nct, t0 + a.tpr);
  auto wanted = [&](int i) { return a.recv[t0 + i] != 0; };
  if (a.probe) {
    // the probe's list is dense: source q's tiles at a base taken from the
    // running total (dem[2R], which bounds the list for K0d and the halo K0b),
    // in any source order -- the exchange's regions are per-source capacities
    __shared__ unsigned pbase;
    const int rc = block_compact(max(t1 - t0, 0), wanted, [](int, int) {});
    if (threadIdx.x == 0) pbase = rc ? atomicAdd(&a.dem[2 * a.R], (unsigned)rc) : 0u;
    __syncthreads();
    int *hl = a.hl + pbase;
    block_compact(max(t1 - t0, 0), wanted, [&](int i, int k) { hl[k] = t0 + i; });
    return;  // (block_compact ends with a barrier: pbase is reused by the next q)
  }
  const int cap = cp.rcap[q];
  int *hl = a.hl + (size_t)cp.hoff[q];
  const int rc = block_compact(max(t1 - t0, 0), wanted, [&](int i, int k) { if (k < cap) hl[k] = t0 + i; });
  for (int k = rc + (int)threadIdx.x; k < cap; k += blockDim.x) hl[k] = -1;
  if (threadIdx.x == 0) {
    a.dem[a.R + q] = (unsigned)rc;
    atomicAdd(&a.dem[2 * a.R], (unsigned)min(rc, cap));
    if (ovf || rc > cap) a.cnt->halo_ovf = 1;
  }
  __syncthreads();  // block_compact's shared words are reused by the next q
}

// The plan.  blockIdx.y < ny: own tiles a0 + y, a0 + y + ny, ... (as K0d's
// row tiles) against every other tile t = blockIdx.x * 256 + lane; y == ny
// (exchange): this rank's requests, and the copy of the gathered boxes into
// tbox_c for K0d; y == ny + 1 (exchange): the other ranks' requests for own
// tiles.  (Ordering the lists in the last workgroup to finish, behind a
// release fence per workgroup, took longer than the separate k_halo_lists
// launch: 16.8 us against 4.5 + 4.4 at 1M, R = 8.)
// plan reuse: every rank's flag word (gathered; the probe: its own) decides
__device__ __forceinline__ bool plan_rebuild(const PlanArgs &a) {
  if (!a.ht.tpr || a.ht.force) return true;
  if (!a.gblk) return *a.ht.myflag != 0u;
  bool any = false;
  for (int q = 0; q < a.R; ++q)
    any |= reinterpret_cast<const unsigned *>(a.gblk + (size_t)q * a.bb + (size_t)a.tpr * sizeof(TileBox))[a.W] != 0u;
  return any;
}

// One launch for the plan AND the lists (round 5: the lists were their own
// launch, ~5 us at 1M R = 8 even when a kept plan made both return at once):
// rows y < npy are the plan's blocks; row y == npy holds one list block per
// source / destination q (blockIdx.x < nlist), which -- when the plan is
// (re)built -- waits until every plan block has counted itself done (`done`,
// a zeroed word behind the plan flags; the plan blocks never wait, so the
// waiting list blocks cannot starve them).  The lists are k_halo_lists_q.
__device__ void halo_lists_block(const ListArgs &a, const HaloCaps &cp, int q, uint8_t *present);
__global__ __launch_bounds__(256) void k_halo_plan(PlanArgs a, int ny, int npy, ListArgs la, HaloCaps cp, int nlist,
                                                   uint8_t *present, unsigned *done) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int na = a.a1 - a.a0, y = blockIdx.y;
  if (y == npy) {  // a list block
    const int q = blockIdx.x;
    if (q >= nlist || (a.ht.tpr && !plan_rebuild(a))) return;  // (the same decision as every plan block)
    if (threadIdx.x == 0) {
      const unsigned np = gridDim.x * (unsigned)npy;
      while (__hip_atomic_load(done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < np) __builtin_amdgcn_s_sleep(2);
    }
    __syncthreads();
    __threadfence();  // (every lane: the plan's stores after the count)
    halo_lists_block(la, cp, q, present);
    return;
  }
  if (a.ht.tpr) {
    const bool rb = plan_rebuild(a);
    if (t == 0 && y == 0) {  // (every block reads the words first: the flag is cleared after this launch)
      a.ht.ctl[0] = rb ? 1ull : 0ull;
    }
    if (!rb) return;
    if (t == 0 && y == 0)
      for (int k = 0; k < a.ndem; ++k) a.dem[k] = 0u;  // the lists kernel writes them next
  }
  // grown boxes when the plan is kept for later detects (symmetric: both sides grow alike)
  auto gr = [&](const TileBox &b) { return a.ht.tpr ? box_grow(b, a.ht.dx, a.ht.ds, a.ht.dv) : b; };
  if (y < ny) {
    if (t < a.nct && !(t >= a.a0 && t < a.a1)) {
      const TileBox b = gr(plan_box(a, t));
      for (int i = y; i < na; i += ny)
        if (boxes_may_interact(gr(a.tbox[a.a0 + i]), b)) {
          a.recv[t] = 1;
          if (a.send) a.send[(size_t)(t / a.tpr) * a.tpr + i] = 1;
        }
    }
  } else if (y == ny) {
    if (a.gblk && t < a.nct && !(t >= a.a0 && t < a.a1)) {
      a.tbox_out[t] = plan_box(a, t);
      if (req_bit(a, a.me, t)) a.recv[t] = 1;
    }
  } else if (a.gblk && t < a.R * na) {  // y == ny + 1: thread = (rank q, own tile i)
    const int q = t / na, i = t - q * na;
    if (q != a.me && req_bit(a, q, a.a0 + i)) a.send[(size_t)q * a.tpr + i] = 1;
  }
  // this block's plan stores, then its count (the list blocks wait for all)
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(done, 1u);
}

// list block q: the lists of source / destination q (halo_lists_q); with
// plan reuse only at a rebuild (decided by every block alike), when it also
// keeps source q's part of the present mask for the detects until the next.
// (The rank's rebuild flag is cleared by K0d, after every block of this
// launch has read it.)
__device__ void halo_lists_block(const ListArgs &a, const HaloCaps &cp, int q, uint8_t *present) {
  if (present) {
    const int t0 = q * a.tpr, t1 = min(a.nct, t0 + a.tpr);
    for (int t = t0 + (int)threadIdx.x; t < t1; t += blockDim.x) present[t] = a.recv[t];
  }
  halo_lists_q(a, cp, q);
}

// rows of the listed own tiles into the send regions: block (slot k, rank q)
__global__ __launch_bounds__(kTile) void k_halo_pack(int n, int me, HaloFields fl, unsigned char *sbuf, HaloCaps cp) {
  const int k = blockIdx.x, q = blockIdx.y;
  if (q == me || k >= cp.scap[q]) return;
  const unsigned *hdr = reinterpret_cast<const unsigned *>(sbuf + cp.soff[q]);
  if (k >= (int)hdr[0]) return;
  const int row = (int)hdr[1 + k] * kTile + (int)threadIdx.x;
  double *dst = reinterpret_cast<double *>(sbuf + cp.soff[q] + halo_hdr_bytes(cp.scap[q]) + (size_t)k * halo_tile_bytes(fl.nf));
  for (int f = 0; f < fl.nf; ++f) dst[f * kTile + threadIdx.x] = row < n ? fl.f[f][row] : 0.0;
}

// ---------------------------------------------------------------- host side
static int nct_of(const Ctx *c) { return (int)((c->n + kTile - 1) / kTile); }
static int tpr_of(const Ctx *c) { return (int)(c->sim_rpr / kTile); }
static int tiles_of(const Ctx *c, int q) {
  const int tpr = tpr_of(c);
  return std::max(0, std::min(nct_of(c), (q + 1) * tpr) - q * tpr);
}
static int64_t cap_at(const Ctx *c, int s, int d) { return c->halo_cap[(size_t)s * c->nranks + d]; }

// region offsets in sender s's buffer (destinations in rank order) and its size
static size_t send_offsets(const Ctx *c, int s, int nf, unsigned long long *off) {
  size_t at = 0;
  for (int d = 0; d < c->nranks; ++d) {
    off[d] = at;
    if (d != s) at += region_bytes((int)cap_at(c, s, d), nf);
  }
  return at;
}

// the tiles this rank holds besides its own: the last plan's (with plan
// reuse the kept plan's, written by k_halo_lists at a rebuild)
const uint8_t *halo_present(const Ctx *c) {
  return c->h_present.p ? (const uint8_t *)c->h_present.p : (const uint8_t *)c->h_plan.p;
}
// the probe's dense halo list: its length on the device (the exchange's list
// has per-source capacity regions, bounded by halo_hl on the host)
const unsigned *halo_list_count(const Ctx *c) {
  return c->halo_mode == 2 ? (const unsigned *)c->h_dem.p + c->halo_tot_word : nullptr;
}

// the plan's buffers: recv [nct] + send [R][tpr] flags, demands ([R] send,
// [R] receive, the total received).  hp: the own-tile
// K0b zeroes them (the regions are recorded there); NULL: memsets here.
static size_t plan_bytes(int nct, int R, int tpr) { return ((size_t)nct + (size_t)R * tpr + 3) / 4 * 4; }
// the merged plan / lists launch's done counter: the word behind the plan flags
static unsigned *plan_done_word(Ctx *c, int nct, int R, int tpr) {
  return (unsigned *)((char *)c->h_plan.p + plan_bytes(nct, R, tpr));
}
static int plan_buffers(Ctx *c, int nct, int R, int tpr, int Rd, HaloPre *hp, bool keep) {
  const size_t pbytes = plan_bytes(nct, R, tpr) + 4, dwords = (size_t)(2 * Rd + 1);  // (+ the done word)
  if (!ensure(c, c->h_plan, pbytes + 64, "halo plan") || !ensure(c, c->h_dem, dwords * 4, "halo demands"))
    return -1;
  if (keep) {  // plan reuse: the kept present mask (k_halo_lists writes it at a rebuild)
    if (!ensure(c, c->h_present, (size_t)nct + 64, "halo present mask")) return -1;
  } else {
    release(c->h_present);
  }
  if (hp) {
    hp->z[0] = (unsigned *)c->h_plan.p;
    hp->zn[0] = (int)((pbytes + 3) / 4);
    hp->z[1] = keep ? nullptr : (unsigned *)c->h_dem.p;  // (kept: zeroed by the plan at a rebuild)
    hp->zn[1] = keep ? 0 : (int)dwords;
  } else {
    BSA_HIP(c, hipMemsetAsync(c->h_plan.p, 0, pbytes, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->h_dem.p, 0, dwords * 4, c->stream));
  }
  return 0;
}

constexpr int kPlanRows = 16;  // k_halo_plan: grid rows over the own tiles
static inline int tile_lo(int64_t rb) { return (int)(rb / kTile); }
// (a rank without rows owns no tile: its clamped rb = n need not be tile-aligned)
static inline int tile_hi(int64_t rb, int64_t re) { return re > rb ? (int)((re + kTile - 1) / kTile) : tile_lo(rb); }

// box block of the exchange: [tpr own tile boxes | W request words | rebuild flag word]
static size_t block_bytes(int tpr, int W) { return ((size_t)tpr * sizeof(TileBox) + (size_t)(W + 1) * 4 + 15) / 16 * 16; }

unsigned *halo_flag_word(Ctx *c) {
  if (c->halo_mode == 2) return c->tpr_ctl.p ? (unsigned *)((unsigned long long *)c->tpr_ctl.p + 5) : nullptr;
  const int nct = nct_of(c), tpr = tpr_of(c), W = (nct + 31) / 32;
  return c->h_blk.p ? (unsigned *)((char *)c->h_blk.p + (size_t)tpr * sizeof(TileBox)) + W : nullptr;
}

int halo_pre(Ctx *c, int64_t rb, int64_t re, HaloPre *hp, const HaloTpr *ht) {
  *hp = HaloPre{};
  const bool keep = ht && ht->tpr;
  const int nct = nct_of(c), a0 = tile_lo(rb), a1 = tile_hi(rb, re), na = a1 - a0;
  if (!ensure(c, c->counters, sizeof(Counters), "counters")) return -1;
  if (c->halo_mode == 2) {  // probe: source blocks of tpr = na tiles, full capacity each
    const int tpr = std::max(na, 1), Rp = (nct + tpr - 1) / tpr;
    if (plan_buffers(c, nct, 1, tpr, Rp, hp, keep)) return -1;
    return ensure(c, c->h_hl, (size_t)Rp * tpr * 4, "halo list") ? 0 : -1;
  }
  const int R = c->nranks, tpr = tpr_of(c), W = (nct + 31) / 32;
  const size_t bb = block_bytes(tpr, W);
  if (!ensure(c, c->h_blk, bb, "halo box block") || !ensure(c, c->h_gblk, bb * R, "halo box blocks")) return -1;
  if (plan_buffers(c, nct, R, tpr, R, hp, keep)) return -1;
  hp->z[2] = (unsigned *)((char *)c->h_blk.p + (size_t)tpr * sizeof(TileBox));  // request words
  hp->zn[2] = W;
  hp->blk = (TileBox *)c->h_blk.p;
  hp->blk_base = a0;
  return 0;
}

// one-GPU plan of the rank owning tiles [a0, a1) (probe and initial capacities):
// every tile's box is in tbox_c; the present mask and the flat list (source
// blocks of tpr tiles, full capacity each) come out.  The buffers were zeroed
// by the caller (plan_buffers).
static int plan_local(Ctx *c, int a0, int a1, int tpr, const HaloTpr *ht) {
  const int nct = nct_of(c), na = a1 - a0;
  const int Rp = (nct + tpr - 1) / tpr;
  c->halo_hl = (int64_t)Rp * tpr;
  c->halo_tot_word = 2 * Rp;
  uint8_t *recv = (uint8_t *)c->h_plan.p;
  const HaloTpr h = ht ? *ht : HaloTpr{};
  PlanArgs pa{nct, tpr, 1, -1, a0, a1, (const TileBox *)c->tbox_c.p, nullptr, 0, nullptr, recv, nullptr,
              0, h, (unsigned *)c->h_dem.p, 2 * Rp + 1};
  ListArgs la{nct, tpr, Rp, -1, a0, a1, 1, recv, nullptr, (int *)c->h_hl.p, nullptr, (unsigned *)c->h_dem.p,
              (Counters *)c->counters.p};
  const int ny = std::max(1, std::min(na, kPlanRows));
  const unsigned gx = (unsigned)std::max((nct + 255) / 256, Rp);
  hipLaunchKernelGGL(k_halo_plan, dim3(gx, (unsigned)(ny + 1)), dim3(256), 0, c->stream, pa, ny, ny, la, HaloCaps{}, Rp,
                     h.tpr ? (uint8_t *)c->h_present.p : (uint8_t *)nullptr, plan_done_word(c, nct, 1, tpr));
  BSA_HIP(c, hipGetLastError());
  return 0;
}

int halo_mid(Ctx *c, int64_t rb, int64_t re, HaloUnpack *hu, HaloTpr *ht, bool hkeep, hipStream_t xs) {
  hu->rbuf = nullptr;
  const int nct = nct_of(c);
  const int a0 = tile_lo(rb), a1 = tile_hi(rb, re), na = a1 - a0;
  if (c->halo_mode == 2) {
    c->halo_fields = 0;
    if (hkeep) {  // HK: the kept plan's dense list (its length stays in h_dem)
      const int tpr = std::max(na, 1), Rp = (nct + tpr - 1) / tpr;
      c->halo_hl = (int64_t)Rp * tpr;
      c->halo_tot_word = 2 * Rp;
      return 0;
    }
    return plan_local(c, a0, a1, std::max(na, 1), ht);
  }
  // ---- exchange mode (several ranks); halo_pre's buffers, zeroed by the own-tile K0b
  const int R = c->nranks, me = c->rank, tpr = tpr_of(c);
  if (R > kHaloMaxRanks) return fail(c, "halo exchange: at most %d ranks", kHaloMaxRanks);
  if ((int64_t)c->halo_cap.size() != (int64_t)R * R) return fail(c, "halo exchange: capacities not set");
  hipStream_t s = c->stream;
  const int W = (nct + 31) / 32;
  const size_t bb = block_bytes(tpr, W);
  // 2. own tile boxes (written by K0b) + request bits -> every rank
  unsigned *req = (unsigned *)((char *)c->h_blk.p + (size_t)tpr * sizeof(TileBox));
  const bool keep = ht && ht->tpr;
  // the fields per halo row fix the regions' layout (the kept send headers sit
  // at its offsets): a change of it is a rebuild on every rank alike (HK: the
  // host checked it before it kept the plan)
  const int nf = (c->simp.winddim == 0 && c->sim_gs_derivable) ? 6 : 8;
  if (hkeep && nf != c->halo_fields) return fail(c, "internal: HK kept the halo plan across a field-count change");
  if (keep && nf != c->halo_fields) ht->force = 1;
  if (!hkeep && c->simp.resume_nav && c->bk_ready && na > 0) {
    hipLaunchKernelGGL(k_halo_req, dim3(64), dim3(256), 0, s, (int)(c->sim_re - c->sim_rb),
                       (const unsigned *)c->bk_rptr.p, (const unsigned *)c->bk_rcol.p, (const unsigned *)c->id2h.p,
                       a0, a1, req, keep ? (const uint8_t *)c->h_present.p : (const uint8_t *)nullptr,
                       keep ? ht->myflag : (unsigned *)nullptr);
    BSA_HIP(c, hipGetLastError());
  }
  if (!hkeep && comm_allgather(c, c->h_blk.p, c->h_gblk.p, bb)) return -1;
  // capacities and offsets of this rank's regions
  HaloCaps cp{};
  size_t roff = 0;
  int hoff = 0, smax = 0;
  const size_t stot = send_offsets(c, me, nf, cp.soff);
  for (int q = 0; q < R; ++q) {
    cp.scap[q] = q == me ? 0 : (int)cap_at(c, me, q);
    cp.rcap[q] = q == me ? 0 : (int)cap_at(c, q, me);
    cp.hoff[q] = hoff;
    cp.roff[q] = roff;
    hoff += cp.rcap[q];
    roff += region_bytes(cp.rcap[q], nf);
    smax = std::max(smax, cp.scap[q]);
  }
  c->halo_hl = hoff;
  c->halo_tot_word = 2 * R;
  c->halo_fields = nf;
  c->halo_tx = (int64_t)stot;
  c->halo_rx = (int64_t)roff;
  if (!ensure(c, c->h_send, std::max<size_t>(stot, 16), "halo send") ||
      !ensure(c, c->h_recv, std::max<size_t>(roff, 16), "halo recv") ||
      !ensure(c, c->h_hl, (size_t)std::max(hoff, 1) * 4, "halo list"))
    return -1;
  // 3. plan + lists, one launch
  uint8_t *recv = (uint8_t *)c->h_plan.p, *sendf = recv + nct;
  const HaloTpr h = ht ? *ht : HaloTpr{};
  PlanArgs pa{nct, tpr, R, me, a0, a1, (const TileBox *)c->tbox_c.p, (const unsigned char *)c->h_gblk.p, bb,
              (TileBox *)c->tbox_c.p, recv, sendf, W, h, (unsigned *)c->h_dem.p, 2 * R + 1};
  ListArgs la{nct, tpr, R, me, a0, a1, 0, recv, sendf, (int *)c->h_hl.p, (unsigned char *)c->h_send.p,
              (unsigned *)c->h_dem.p, (Counters *)c->counters.p};
  const int ny = std::max(1, std::min(na, kPlanRows));
  const unsigned gx = (unsigned)std::max((std::max(nct, R * na) + 255) / 256, R);
  if (!hkeep) {  // (HK: the kept plan's send headers and halo list stay as they are)
    hipLaunchKernelGGL(k_halo_plan, dim3(gx, (unsigned)(ny + 3)), dim3(256), 0, s, pa, ny, ny + 2, la, cp, R,
                       h.tpr ? (uint8_t *)c->h_present.p : (uint8_t *)nullptr, plan_done_word(c, nct, R, tpr));
    BSA_HIP(c, hipGetLastError());
  }
  HaloFields fl{};
  DevBuf *src[8] = {&c->own[0], &c->own[1], &c->own[2], &c->own[3], &c->own[4], &c->own[5], &c->s_gse, &c->s_gsn};
  for (int f = 0; f < 8; ++f) fl.f[f] = (double *)src[f]->p;
  fl.nf = nf;
  // 4. pack, exchange (the halo K0b unpacks: hu)
  if (smax > 0) {
    hipLaunchKernelGGL(k_halo_pack, dim3((unsigned)smax, (unsigned)R), dim3(kTile), 0, s, (int)c->n, me, fl,
                       (unsigned char *)c->h_send.p, cp);
    BSA_HIP(c, hipGetLastError());
  }
  std::vector<size_t> slen(R), rlen(R), rof(R), peer(R);
  for (int q = 0; q < R; ++q) {
    slen[q] = q == me ? 0 : region_bytes(cp.scap[q], nf);
    rlen[q] = q == me ? 0 : region_bytes(cp.rcap[q], nf);
    rof[q] = cp.roff[q];
    unsigned long long po[kHaloMaxRanks];
    send_offsets(c, q, nf, po);  // where rank q's region for this rank starts in q's buffer
    peer[q] = po[me];
  }
  std::vector<size_t> sof(R);
  for (int q = 0; q < R; ++q) sof[q] = cp.soff[q];
  if (xs) {  // halo overlap: the send / recv on xs (the collective runs on whatever stream c->stream names)
    BSA_HIP(c, hipEventRecord(c->ov_ev[0], s));
    BSA_HIP(c, hipStreamWaitEvent(xs, c->ov_ev[0], 0));
    std::swap(c->stream, xs);
    const int rc = comm_halo(c, c->h_send.p, sof.data(), slen.data(), stot, c->h_recv.p, rof.data(), rlen.data(),
                             peer.data());
    std::swap(c->stream, xs);
    if (rc) return -1;
  } else if (comm_halo(c, c->h_send.p, sof.data(), slen.data(), stot, c->h_recv.p, rof.data(), rlen.data(),
                       peer.data())) {
    return -1;
  }
  hu->rbuf = (const unsigned char *)c->h_recv.p;
  hu->cp = cp;
  hu->fl = fl;
  hu->R = R;
  hu->n = (int)c->n;
  return 0;
}

// Exact initial capacities: at bsa_sim_init every rank holds the whole state,
// so each computes every rank's plan itself (the same numbers on all ranks).
int halo_init_caps(Ctx *c) {
  const int R = c->nranks, tpr = tpr_of(c), nct = nct_of(c);
  c->halo_cap.assign((size_t)R * R, 0);
  c->halo_grows = 0;
  if (R <= 1) return 0;
  if (prep_all_tiles(c, c->simp.rpz, c->simp.hpz, c->simp.tla)) return -1;
  std::vector<uint8_t> recv((size_t)nct);
  for (int q = 0; q < R; ++q) {
    const int a0 = q * tpr, a1 = a0 + tiles_of(c, q);
    const int Rp = (nct + tpr - 1) / tpr;
    // (with plan reuse every plan is made on grown boxes: the capacities too)
    HaloTpr ht{c->tpr_on ? 1 : 0, 1, c->tpr_dx, c->tpr_ds, c->tpr_dv, nullptr, nullptr};
    if (ht.tpr) {
      const bool fresh = !c->tpr_ctl.p;  // (ensure does not zero: the build / detect counters start at 0)
      if (!ensure(c, c->tpr_ctl, 64, "tile-pair list control")) return -1;
      if (fresh) BSA_HIP(c, hipMemsetAsync(c->tpr_ctl.p, 0, 64, c->stream));
      ht.ctl = (unsigned long long *)c->tpr_ctl.p;
      ht.myflag = (unsigned *)(ht.ctl + 5);
    }
    if (plan_buffers(c, nct, 1, tpr, Rp, nullptr, false) || !ensure(c, c->h_hl, (size_t)Rp * tpr * 4, "halo list") ||
        plan_local(c, a0, a1, tpr, ht.tpr ? &ht : nullptr))
      return -1;
    BSA_HIP(c, hipMemcpyAsync(recv.data(), c->h_plan.p, (size_t)nct, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    for (int t = 0; t < nct; ++t)
      if (recv[(size_t)t]) c->halo_cap[(size_t)(t / tpr) * R + q]++;
  }
  for (int sd = 0; sd < R; ++sd)
    for (int q = 0; q < R; ++q) {
      int64_t &m = c->halo_cap[(size_t)sd * R + q];
      if (m) m = std::min<int64_t>(m + m / 4 + 2, tiles_of(c, sd));
    }
  c->halo_cap_gen++;  // (every rank, bsa_sim_init): the next exchange re-checks the region layout
  return 0;
}

// After an aborted step (every rank, collective): the demands of this rank's
// plan are max-all-reduced into an R x R matrix; capacities below it grow.
int halo_grow(Ctx *c) {
  const int R = c->nranks, me = c->rank;
  if (R <= 1 || (int64_t)c->halo_cap.size() != (int64_t)R * R) return 0;
  std::vector<unsigned> dem((size_t)2 * R + 1, 0u);
  if (c->h_dem.p) {
    BSA_HIP(c, hipMemcpyAsync(dem.data(), c->h_dem.p, dem.size() * 4, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
  }
  std::vector<double> m((size_t)R * R, 0.0);
  for (int q = 0; q < R; ++q) {
    if (q == me) continue;
    m[(size_t)me * R + q] = dem[(size_t)q];      // what this rank must send to q
    m[(size_t)q * R + me] = dem[(size_t)R + q];  // what it must receive from q
  }
  if (comm_allreduce_host(c, m.data(), R * R, true)) return -1;
  bool grew = false;
  for (int sd = 0; sd < R; ++sd)
    for (int q = 0; q < R; ++q) {
      int64_t &cap = c->halo_cap[(size_t)sd * R + q];
      const int64_t need = (int64_t)m[(size_t)sd * R + q];
      if (need > cap) {
        cap = std::min<int64_t>(std::max(2 * cap, need + need / 4 + 2), tiles_of(c, sd));
        grew = true;
      }
    }
  if (grew) {
    c->halo_grows++;
    c->halo_cap_gen++;  // (collective: the same decision on every rank)
  }
  return 0;
}

void halo_release(Ctx *c) {
  DevBuf *all[] = {&c->h_blk, &c->h_gblk, &c->h_plan, &c->h_lists, &c->h_send, &c->h_recv, &c->h_hl, &c->h_dem,
                   &c->h_present};
  for (auto *b : all) release(*b);
  c->halo_cap.clear();
  c->halo_hl = 0;
}

}  // namespace bsa
