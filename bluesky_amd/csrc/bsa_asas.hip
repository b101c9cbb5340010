// ASAS.update bookkeeping and ResumeNav on the device (asas.py:409-504) for
// the resident sim step, opt-in (bsa_sim_params.resume_nav).
//
// resopairs is kept as CSR over the rank's own rows (row = idx1 - rb, sorted
// idx2 per row).  Per CD call, after K3:
//   before MVP (bk_count; MVP changes none of the state these read):
//   k_bk_count   one lane per row: merge the row's resopairs with the row's
//                new confpairs (K2 output, sorted), evaluate ResumeNav's
//                past-CPA / horizontal-LoS / bouncing test per pair
//                (asas.py:424-452), count the kept pairs
//   scan         kept counts -> next CSR (single-pass scan_excl)
//   k_bk_check   next CSR larger than its buffer -> gate bit 1: the step
//                aborts before MVP touches asas state (all ranks, through the
//                gate all-reduce); the host grows the buffer and retries
//   after MVP (bk_apply):
//   k_bk_write   same merge + test, write the kept pairs and asas.active
//                (true iff any of the row's pairs is kept; rows without
//                resopairs keep their value, as in the reference)
//   k_bk_unique  |confpairs_unique|, |lospairs_unique| and the growth of
//                confpairs_all / lospairs_all (asas.py:494-502): pair (i, j)
//                is the representative of {i, j} when i < j or (j, i) is not a
//                pair; it is new when neither (i, j) nor (j, i) was a pair of
//                the previous call.  One rank: on the K2 CSR.  Several ranks
//                (k_bk_unique_g): the sets are global, so every rank packs its
//                pair keys (k_bk_pack, before the gate: a full key buffer
//                aborts the step like a resopairs overflow), one all-gather
//                replicates all ranks' blocks -- concatenated in rank order
//                they are the global row-major lists -- and every rank counts
//                the global sets itself (identical counts on all ranks)
//   k_bk_commit  copy the next CSR and this call's pair lists over the
//                persistent ones (several ranks: the gathered key blocks)
// Every kernel is a no-op once the step batch is aborted (sticky flag), so a
// retried step finds the bookkeeping as it was at the step's start.  The
// reference iterates a Python set in ResumeNav, so an aircraft whose pairs
// disagree ends with whichever pair its hash order visits last; the device
// (and oracle/asas.py) use "active iff any kept pair" (DESIGN.md 3.8).
#include <hipcub/hipcub.hpp>

#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

struct BkIn {
  int rb, nrows;
  const unsigned *rptr;    // resopairs CSR (persistent), nrows + 1
  const unsigned *rcol;
  const unsigned *cptr;    // this call's conflict rows: K2 row offsets, nrows + 1
  const int *ccol;         // K2 cj (original column index, ascending per row)
  const double *lat, *lon, *gse, *gsn, *trk;  // full-N state (home order)
  const unsigned *id2h;    // aircraft index -> home (the CSR columns are indices)
  double R, Rm;
  const unsigned long long *gate;
  const unsigned *sticky;
  unsigned *cnt;           // kept per row (count pass)
  const unsigned *nptr;    // next CSR pointers (write pass)
  unsigned *ncol;
  uint8_t *active;         // full-N
  uint8_t *dropped;        // full-N (home order) or NULL: the row dropped a pair this call
  unsigned long long *stats;
};

__device__ __forceinline__ bool bk_aborted(const unsigned long long *gate, const unsigned *sticky) {
  return sticky[0] != 0 || gate[0] >= kGateOverflow;
}

// ResumeNav's decision for resopair (i, j), asas.py:424-452.  j == kDangling:
// the intruder was deleted (bsa_sim_delete) -- idx2 < 0 switches ASAS off for
// the ownship and drops the pair (asas.py:454-468)
__device__ __forceinline__ bool bk_keep(const BkIn &in, int i, int j) {
  if ((unsigned)j == kDangling) return false;
  j = (int)in.id2h[j];  // i: home row, j: the intruder's index
  const double re = 6371000.;
  const double d0 = re * (((in.lon[j] - in.lon[i]) * kD2R) * cos(0.5 * ((in.lat[j] + in.lat[i]) * kD2R)));
  const double d1 = re * ((in.lat[j] - in.lat[i]) * kD2R);
  const double v0 = in.gse[j] - in.gse[i], v1 = in.gsn[j] - in.gsn[i];
  const bool past_cpa = d0 * v0 + d1 * v1 > 0.0;
  const double hdist = sqrt(d0 * d0 + d1 * d1);
  const bool hor_los = hdist < in.R;
  const bool bouncing = fabs(in.trk[i] - in.trk[j]) < 30.0 && hdist < in.Rm;
  return !past_cpa || hor_los || bouncing;
}

// walk the sorted union of row r's resopairs and new confpairs
template <typename F>
__device__ __forceinline__ void bk_merge(const BkIn &in, int r, F f) {
  unsigned a = in.rptr[r], ae = in.rptr[r + 1];
  unsigned b = in.cptr[r], be = in.cptr[r + 1];
  while (a < ae || b < be) {
    unsigned j;
    if (b >= be || (a < ae && in.rcol[a] < (unsigned)in.ccol[b])) {
      j = in.rcol[a++];
    } else if (a >= ae || (unsigned)in.ccol[b] < in.rcol[a]) {
      j = (unsigned)in.ccol[b++];
    } else {  // in both
      j = in.rcol[a++];
      ++b;
    }
    f(j);
  }
}

__global__ __launch_bounds__(256) void k_bk_count(BkIn in) {
  if (bk_aborted(in.gate, in.sticky)) return;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > in.nrows) return;
  unsigned kept = 0;
  if (r < in.nrows) {
    const int i = in.rb + r;
    bk_merge(in, r, [&](unsigned j) { kept += bk_keep(in, i, (int)j) ? 1u : 0u; });
  }
  in.cnt[r] = kept;  // cnt[nrows] = 0: the exclusive scan's last entry is the total
}

__global__ void k_bk_check(int nrows, const unsigned *nptr, unsigned long long ncap, unsigned long long *gate,
                           const unsigned *sticky, unsigned long long *demand) {
  if (bk_aborted(gate, sticky)) return;
  const unsigned long long total = nptr[nrows];
  if (total > ncap) {
    gate[0] = kGateBkOverflow;
    *demand = total > *demand ? total : *demand;
  }
}

__global__ __launch_bounds__(256) void k_bk_write(BkIn in) {
  if (bk_aborted(in.gate, in.sticky)) return;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r == 0) {
    in.stats[0] = in.nptr[in.nrows];
    in.stats[1] = 0;  // per-call unique counts (k_bk_unique adds)
    in.stats[2] = 0;
  }
  if (r >= in.nrows) return;
  const int i = in.rb + r;
  unsigned pos = in.nptr[r];
  bool any = false, seen = false, drop = false;
  bk_merge(in, r, [&](unsigned j) {
    seen = true;
    if (bk_keep(in, i, (int)j)) {
      in.ncol[pos++] = j;
      any = true;
    } else {
      drop = true;  // asas.py:454-468: ASAS off, waypoint recovery (route.direct) for the ownship
    }
  });
  if (seen) in.active[i] = any ? 1 : 0;
  if (in.dropped) in.dropped[i] = drop ? 1 : 0;
}

// is (r, c) in the CSR (ptr over rows 0.., ascending cols)?
__device__ __forceinline__ bool csr_has(const unsigned *ptr, const int *col, int r, int c) {
  const unsigned e = ptr[r + 1];
  unsigned lo = ptr[r], hi = e;
  while (lo < hi) {
    const unsigned mid = (lo + hi) >> 1;
    if (col[mid] < c) lo = mid + 1; else hi = mid;
  }
  return lo < e && col[lo] == c;
}

struct BkUniq {
  const int *ci, *cj;         // this call's pairs (row-major): ci home rows, cj indices
  const unsigned *h2id, *id2h;
  const unsigned *ptr;        // this call's row offsets (conf: rowoff; los: lptr)
  const unsigned *np;         // device pair count
  const unsigned *pptr;       // previous call's CSR
  const int *pcol;
  unsigned long long *uniq, *all;
};

// per-workgroup sums of two counts, then ONE atomic each per workgroup (a
// per-wave atomic on one word serialises at ~12 ns each)
__device__ __forceinline__ void block_add2(unsigned long long a, unsigned long long b, unsigned long long *pa,
                                           unsigned long long *pb) {
  __shared__ unsigned long long s[2][4];
  const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    s[0][w] = a;
    s[1][w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long ta = 0, tb = 0;
    for (unsigned q = 0; q < blockDim.x / 64; ++q) {
      ta += s[0][q];
      tb += s[1][q];
    }
    if (ta) atomicAdd(pa, ta);
    if (tb) atomicAdd(pb, tb);
  }
}

__global__ __launch_bounds__(256) void k_bk_unique(BkUniq u, const unsigned long long *gate, const unsigned *sticky) {
  if (bk_aborted(gate, sticky)) return;
  const unsigned P = *u.np;
  const unsigned lane = threadIdx.x & 63;
  unsigned long long nrep = 0, nfresh = 0;  // this wave's counts (lane 0)
  for (unsigned x = blockIdx.x * blockDim.x + threadIdx.x; x - lane < P; x += gridDim.x * blockDim.x) {
    bool rep = false, fresh = false;
    if (x < P) {
      // (i, j) in home-row / index terms; the representative rule compares indices
      const int i = u.ci[x], j = u.cj[x];
      const int ii = (int)u.h2id[i], jh = (int)u.id2h[j];
      rep = ii < j || !csr_has(u.ptr, u.cj, jh, ii);
      if (rep) fresh = !(csr_has(u.pptr, u.pcol, i, j) || csr_has(u.pptr, u.pcol, jh, ii));
    }
    const unsigned long long mr = __ballot(rep), mf = __ballot(fresh);
    nrep += (unsigned long long)__popcll(mr);
    nfresh += (unsigned long long)__popcll(mf);
  }
  block_add2(nrep, nfresh, u.uniq, u.all);
}

// LoS row pointers from K2's offsets: lptr[r] = rowoff[nrows + 1 + r] - P
__global__ __launch_bounds__(256) void k_bk_lptr(int nrows, const unsigned *rowoff, unsigned *lptr,
                                                 const unsigned long long *gate, const unsigned *sticky) {
  if (bk_aborted(gate, sticky)) return;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r <= nrows) lptr[r] = rowoff[nrows + 1 + r] - rowoff[nrows];
}

// next CSR -> persistent; this call's pair CSRs -> "previous"
struct BkCommit {
  int nrows;
  const unsigned *nptr, *ncol;
  unsigned *rptr, *rcol;
  const unsigned *cptr, *lptr;   // this call (conf rowoff, los pointers)
  const int *ccol, *lcol;
  unsigned *pcptr, *plptr;
  int *pccol, *plcol;
  int uniq;                      // keep the previous-call lists (one rank)
};

__global__ __launch_bounds__(256) void k_bk_commit(BkCommit m, const unsigned long long *gate,
                                                   const unsigned *sticky) {
  if (bk_aborted(gate, sticky)) return;
  const unsigned R = m.nptr[m.nrows];
  const unsigned P = m.uniq ? m.cptr[m.nrows] : 0u, L = m.uniq ? m.lptr[m.nrows] : 0u;
  const unsigned stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
  for (unsigned k = t0; k <= (unsigned)m.nrows; k += stride) {
    m.rptr[k] = m.nptr[k];
    if (m.uniq) {
      m.pcptr[k] = m.cptr[k];
      m.plptr[k] = m.lptr[k];
    }
  }
  for (unsigned k = t0; k < R; k += stride) m.rcol[k] = m.ncol[k];
  for (unsigned k = t0; k < P; k += stride) m.pccol[k] = m.ccol[k];
  for (unsigned k = t0; k < L; k += stride) m.plcol[k] = m.lcol[k];
}


// ---- several ranks: global pair-key blocks.  Block of rank q (W words):
// [0] conflict pairs Pc, [1] LoS pairs Pl, then Pc conflict keys and Pl LoS
// keys, key = i << 32 | j, ascending (rows of rank q, row-major).
__global__ __launch_bounds__(256) void k_bk_pack(int nrows, const unsigned *rowoff, const int *ci, const int *cj,
                                                 const int *li, const int *lj, unsigned long long W,
                                                 unsigned long long *blk, unsigned long long *gate,
                                                 const unsigned *sticky, unsigned long long *demand) {
  if (bk_aborted(gate, sticky)) return;
  // (a rank without rows has no K2 offsets: no pairs)
  const unsigned long long Pc = nrows ? rowoff[nrows] : 0, Pl = nrows ? rowoff[2 * nrows + 1] - rowoff[nrows + 1] : 0;
  const unsigned long long need = 2 + Pc + Pl;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
  if (need > W) {
    if (t == 0) {
      gate[0] = kGateBkOverflow;
      atomicMax(demand, need);
    }
    return;
  }
  if (t == 0) {
    blk[0] = Pc;
    blk[1] = Pl;
  }
  for (unsigned long long x = t; x < Pc; x += stride)
    blk[2 + x] = (unsigned long long)(unsigned)ci[x] << 32 | (unsigned)cj[x];
  for (unsigned long long x = t; x < Pl; x += stride)
    blk[2 + Pc + x] = (unsigned long long)(unsigned)li[x] << 32 | (unsigned)lj[x];
}

struct KeyBlocks {
  const unsigned long long *cur, *prev;  // nranks x W words each
  unsigned long long W;
  int nranks, rpr;                       // rows per rank: home row i lives in block i / rpr
  const unsigned *h2id, *id2h;
};

// is (i, j) a pair of the global list (los = 0: conflicts, 1: LoS)?
__device__ __forceinline__ bool key_has(const unsigned long long *blocks, unsigned long long W, int rpr, int los,
                                        unsigned i, unsigned j) {
  const unsigned long long *b = blocks + (size_t)(i / (unsigned)rpr) * W;
  const unsigned long long Pc = b[0], Pl = b[1];
  const unsigned long long *k = b + 2 + (los ? Pc : 0);
  unsigned long long lo = 0, hi = los ? Pl : Pc;
  const unsigned long long key = (unsigned long long)i << 32 | j;
  while (lo < hi) {
    const unsigned long long mid = (lo + hi) >> 1;
    if (k[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo < (los ? Pl : Pc) && k[lo] == key;
}

// blockIdx.y = rank block, blockIdx.z = 0 conflicts / 1 LoS
__global__ __launch_bounds__(256) void k_bk_unique_g(KeyBlocks kb, unsigned long long *st,
                                                     const unsigned long long *gate, const unsigned *sticky) {
  if (bk_aborted(gate, sticky)) return;
  const int los = blockIdx.z;
  const unsigned long long *b = kb.cur + (size_t)blockIdx.y * kb.W;
  const unsigned long long P = los ? b[1] : b[0];
  const unsigned long long *keys = b + 2 + (los ? b[0] : 0);
  const unsigned lane = threadIdx.x & 63;
  unsigned long long nrep = 0, nfresh = 0;
  for (unsigned long long x = blockIdx.x * blockDim.x + threadIdx.x; x - lane < P;
       x += (unsigned long long)gridDim.x * blockDim.x) {
    bool rep = false, fresh = false;
    if (x < P) {
      // key = home row << 32 | index; the representative rule compares indices
      const unsigned i = (unsigned)(keys[x] >> 32), j = (unsigned)keys[x];
      const unsigned ii = kb.h2id[i], jh = kb.id2h[j];
      rep = ii < j || !key_has(kb.cur, kb.W, kb.rpr, los, jh, ii);
      if (rep) fresh = !(key_has(kb.prev, kb.W, kb.rpr, los, i, j) || key_has(kb.prev, kb.W, kb.rpr, los, jh, ii));
    }
    const unsigned long long mr = __ballot(rep), mf = __ballot(fresh);
    nrep += (unsigned long long)__popcll(mr);
    nfresh += (unsigned long long)__popcll(mf);
  }
  block_add2(nrep, nfresh, st + 1 + los, st + 3 + los);
}

__global__ __launch_bounds__(256) void k_bk_copy_keys(unsigned long long words, const unsigned long long *src,
                                                      unsigned long long *dst, const unsigned long long *gate,
                                                      const unsigned *sticky) {
  if (bk_aborted(gate, sticky)) return;
  for (unsigned long long k = blockIdx.x * blockDim.x + threadIdx.x; k < words;
       k += (unsigned long long)gridDim.x * blockDim.x)
    dst[k] = src[k];
}

static BkIn bk_in(Ctx *c, const BkDev &d) {
  BkIn in;
  in.rb = (int)c->last_rb;
  in.nrows = (int)(c->last_re - c->last_rb);
  in.rptr = (const unsigned *)c->bk_rptr.p;
  in.rcol = (const unsigned *)c->bk_rcol.p;
  in.cptr = (const unsigned *)c->rowoff.p;
  in.ccol = (const int *)c->out_cj.p;
  in.lat = d.lat;
  in.lon = d.lon;
  in.gse = d.gse;
  in.gsn = d.gsn;
  in.trk = d.trk;
  in.id2h = d.id2h;
  in.R = c->simp.rpz;        // asas.R
  in.Rm = c->simp.mvp.Rm;    // asas.R * asas.mar (MVP.py:24)
  in.gate = d.gate;
  in.sticky = d.sticky;
  in.cnt = (unsigned *)c->bk_cnt.p;
  in.nptr = (const unsigned *)c->bk_nptr.p;
  in.ncol = (unsigned *)c->bk_ncol.p;
  in.active = d.active;
  in.dropped = d.dropped;
  in.stats = (unsigned long long *)c->bk_stats.p;
  return in;
}

// capacity of the resopairs CSR (an overflow aborts the step and regrows)
static unsigned long long bk_ncap(Ctx *c) { return c->bk_cap; }

int bk_count(Ctx *c, const BkDev &d) {
  const int64_t nrows = std::max<int64_t>(c->last_re - c->last_rb, 0), n = c->n;
  // a rank without rows still takes part in the key all-gather (several ranks)
  if (nrows == 0 && !comm_multi(c)) return 0;
  if (c->bk_cap == 0) c->bk_cap = std::max<unsigned long long>(c->cand_cap, 1 << 16);
  const unsigned long long ncap = bk_ncap(c);
  const size_t lcap = (size_t)std::max(c->cand_cap, c->los_cap) * 4;
  if (!ensure_keep(c, c->bk_rptr, (size_t)(nrows + 1) * 4, "resopairs rows") ||
      !ensure_keep(c, c->bk_rcol, (size_t)ncap * 4, "resopairs") ||
      !ensure(c, c->bk_nptr, (size_t)(nrows + 1) * 4, "resopairs next rows") ||
      !ensure(c, c->bk_ncol, (size_t)ncap * 4, "resopairs next") ||
      !ensure(c, c->bk_cnt, (size_t)(nrows + 1) * 4, "resopairs counts") ||
      !ensure(c, c->bk_lptr, (size_t)(nrows + 1) * 4, "los rows") ||
      !ensure_keep(c, c->bk_pcptr, (size_t)(n + 1) * 4, "previous conflict rows") ||
      !ensure_keep(c, c->bk_plptr, (size_t)(n + 1) * 4, "previous los rows") ||
      !ensure_keep(c, c->bk_pccol, (size_t)c->cand_cap * 4, "previous conflicts") ||
      !ensure_keep(c, c->bk_plcol, lcap, "previous los") ||
      !ensure_keep(c, c->bk_stats, 8 * 8, "bookkeeping stats"))
    return -1;
  const bool multi = comm_multi(c);
  if (multi) {  // global unique-pair sets: this rank's key block + all ranks' (this and the previous call)
    if (c->bk_kw == 0) c->bk_kw = 1 << 16;
    const size_t blk = (size_t)c->bk_kw * 8, all = blk * c->nranks;
    if (c->bk_ready && c->bk_kw_alloc && c->bk_kw != c->bk_kw_alloc) {
      // key blocks regrown after an overflow: re-lay the previous call's blocks out at the new width
      DevBuf nb;
      if (!ensure(c, nb, all, "previous gathered pair keys")) return -1;
      BSA_HIP(c, hipMemsetAsync(nb.p, 0, all, c->stream));
      BSA_HIP(c, hipMemcpy2DAsync(nb.p, blk, c->bk_kprev.p, (size_t)c->bk_kw_alloc * 8,
                                  (size_t)c->bk_kw_alloc * 8, c->nranks, hipMemcpyDeviceToDevice, c->stream));
      BSA_HIP(c, hipStreamSynchronize(c->stream));
      release(c->bk_kprev);
      c->bk_kprev = nb;
    }
    if (!ensure(c, c->bk_ksend, blk, "pair key block") || !ensure(c, c->bk_kcur, all, "gathered pair keys") ||
        !ensure_keep(c, c->bk_kprev, all, "previous gathered pair keys"))
      return -1;
    c->bk_kw_alloc = c->bk_kw;
  }
  if (!c->bk_ready) {  // empty sets
    BSA_HIP(c, hipMemsetAsync(c->bk_rptr.p, 0, (size_t)(nrows + 1) * 4, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->bk_pcptr.p, 0, (size_t)(n + 1) * 4, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->bk_plptr.p, 0, (size_t)(n + 1) * 4, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->bk_stats.p, 0, 8 * 8, c->stream));
    if (multi) BSA_HIP(c, hipMemsetAsync(c->bk_kprev.p, 0, (size_t)c->bk_kw * 8 * c->nranks, c->stream));
    c->bk_ready = true;
  }
  const BkIn in = bk_in(c, d);
  hipLaunchKernelGGL(k_bk_count, dim3((unsigned)((nrows + 1 + 255) / 256)), dim3(256), 0, c->stream, in);
  BSA_HIP(c, hipGetLastError());
  if (scan_excl(c, (const unsigned *)c->bk_cnt.p, (unsigned *)c->bk_nptr.p, (int)(nrows + 1))) return -1;
  hipLaunchKernelGGL(k_bk_check, dim3(1), dim3(1), 0, c->stream, (int)nrows, (const unsigned *)c->bk_nptr.p,
                     ncap, d.gate, (const unsigned *)d.sticky, d.demand);
  BSA_HIP(c, hipGetLastError());
  if (multi) {
    hipLaunchKernelGGL(k_bk_pack, dim3(256), dim3(256), 0, c->stream, (int)nrows, (const unsigned *)c->rowoff.p,
                       (const int *)c->out_ci.p, (const int *)c->out_cj.p, (const int *)c->out_li.p,
                       (const int *)c->out_lj.p, (unsigned long long)c->bk_kw,
                       (unsigned long long *)c->bk_ksend.p, d.gate, (const unsigned *)d.sticky, d.kdemand);
    BSA_HIP(c, hipGetLastError());
  }
  return 0;
}

int bk_apply(Ctx *c, const BkDev &d) {
  const int64_t nrows = std::max<int64_t>(c->last_re - c->last_rb, 0);
  if (nrows == 0 && !comm_multi(c)) return 0;
  const bool multi = comm_multi(c), uniq = !multi;
  const BkIn in = bk_in(c, d);
  const unsigned nb = (unsigned)std::max<int64_t>((nrows + 255) / 256, 1);  // block 0 resets the per-call counts
  hipLaunchKernelGGL(k_bk_write, dim3(nb), dim3(256), 0, c->stream, in);
  BSA_HIP(c, hipGetLastError());
  hipLaunchKernelGGL(k_bk_lptr, dim3((unsigned)((nrows + 1 + 255) / 256)), dim3(256), 0, c->stream,
                     (int)nrows, (const unsigned *)c->rowoff.p, (unsigned *)c->bk_lptr.p, d.gate,
                     (const unsigned *)d.sticky);
  BSA_HIP(c, hipGetLastError());
  unsigned long long *st = (unsigned long long *)c->bk_stats.p;
  if (uniq) {
    BkUniq u;
    u.ci = (const int *)c->out_ci.p;
    u.cj = (const int *)c->out_cj.p;
    u.ptr = (const unsigned *)c->rowoff.p;
    u.np = (const unsigned *)c->rowoff.p + nrows;
    u.pptr = (const unsigned *)c->bk_pcptr.p;
    u.pcol = (const int *)c->bk_pccol.p;
    u.h2id = d.h2id;
    u.id2h = d.id2h;
    u.uniq = st + 1;
    u.all = st + 3;
    hipLaunchKernelGGL(k_bk_unique, dim3(256), dim3(256), 0, c->stream, u, (const unsigned long long *)d.gate,
                       (const unsigned *)d.sticky);
    u.ci = (const int *)c->out_li.p;
    u.cj = (const int *)c->out_lj.p;
    u.ptr = (const unsigned *)c->bk_lptr.p;
    u.np = (const unsigned *)c->bk_lptr.p + nrows;
    u.pptr = (const unsigned *)c->bk_plptr.p;
    u.pcol = (const int *)c->bk_plcol.p;
    u.uniq = st + 2;
    u.all = st + 4;
    hipLaunchKernelGGL(k_bk_unique, dim3(256), dim3(256), 0, c->stream, u, (const unsigned long long *)d.gate,
                       (const unsigned *)d.sticky);
    BSA_HIP(c, hipGetLastError());
  } else {
    // every rank's key block (stream-ordered after k_bk_pack and the gate)
    const size_t blk = (size_t)c->bk_kw * 8;
    if (comm_allgather(c, c->bk_ksend.p, c->bk_kcur.p, blk)) return -1;
    KeyBlocks kb{(const unsigned long long *)c->bk_kcur.p, (const unsigned long long *)c->bk_kprev.p,
                 (unsigned long long)c->bk_kw, c->nranks, (int)c->sim_rpr, d.h2id, d.id2h};
    hipLaunchKernelGGL(k_bk_unique_g, dim3(64, c->nranks, 2), dim3(256), 0, c->stream, kb, st,
                       (const unsigned long long *)d.gate, (const unsigned *)d.sticky);
    BSA_HIP(c, hipGetLastError());
    hipLaunchKernelGGL(k_bk_copy_keys, dim3(256), dim3(256), 0, c->stream,
                       (unsigned long long)c->bk_kw * c->nranks, (const unsigned long long *)c->bk_kcur.p,
                       (unsigned long long *)c->bk_kprev.p, (const unsigned long long *)d.gate,
                       (const unsigned *)d.sticky);
    BSA_HIP(c, hipGetLastError());
  }
  BkCommit m;
  m.nrows = (int)nrows;
  m.nptr = (const unsigned *)c->bk_nptr.p;
  m.ncol = (const unsigned *)c->bk_ncol.p;
  m.rptr = (unsigned *)c->bk_rptr.p;
  m.rcol = (unsigned *)c->bk_rcol.p;
  m.cptr = (const unsigned *)c->rowoff.p;
  m.lptr = (const unsigned *)c->bk_lptr.p;
  m.ccol = (const int *)c->out_cj.p;
  m.lcol = (const int *)c->out_lj.p;
  m.pcptr = (unsigned *)c->bk_pcptr.p;
  m.plptr = (unsigned *)c->bk_plptr.p;
  m.pccol = (int *)c->bk_pccol.p;
  m.plcol = (int *)c->bk_plcol.p;
  m.uniq = uniq ? 1 : 0;
  hipLaunchKernelGGL(k_bk_commit, dim3(512), dim3(256), 0, c->stream, m, (const unsigned long long *)d.gate,
                     (const unsigned *)d.sticky);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

void bk_release(Ctx *c) {
  DevBuf *all[] = {&c->bk_rptr, &c->bk_rcol, &c->bk_nptr, &c->bk_ncol, &c->bk_cnt, &c->bk_lptr,
                   &c->bk_pcptr, &c->bk_plptr, &c->bk_pccol, &c->bk_plcol, &c->bk_stats, &c->bk_tmp,
                   &c->bk_ksend, &c->bk_kcur, &c->bk_kprev};
  for (auto *b : all) release(*b);
  c->bk_ready = false;
  c->bk_cap = 0;
  c->bk_kw = c->bk_kw_alloc = 0;
}

}  // namespace bsa
