// TrafficArrays create / delete on the GPU-resident sim:
// Traffic.create (traffic.py:192-312) appends aircraft to every per-aircraft
// array and ASAS.create (asas.py:402-407) starts their asas.trk / tas / alt at
// the traffic's values; Traffic.delete (traffic.py:364-378 ->
// trafficarrays.py:99-117) removes indices from every array with np.delete,
// so later aircraft shift down.  The ASAS bookkeeping of the reference is
// keyed by callsign and is NOT touched by either (asas.py:409-504):
//   * a resopair whose ownship was deleted is dropped at the next ResumeNav
//     (idx1 < 0, asas.py:421-423) -- here at once (nothing reads it before);
//   * a resopair whose intruder was deleted stays until the next ResumeNav,
//     which switches ASAS off for the ownship and drops it (idx2 < 0,
//     asas.py:454-468) -- here its column becomes kDangling, which k_bk_*
//     treat exactly so;
//   * the previous call's unique pair sets keep deleted callsigns, which can
//     never match a later pair -- here those pairs are dropped.
// Index remapping keeps every CSR row and column order (np.delete keeps the
// order of the remaining aircraft), so no re-sort is needed.  Limitation: a
// callsign deleted and re-created before the next CD call counts as a new
// aircraft here, while the reference's id-keyed sets would match it.
// Several ranks: every rank completes its replicas first, the change is the
// same computation everywhere, and the rows (with their bookkeeping) are
// re-partitioned over the new n (multi_begin / multi_end below).
#include <algorithm>
#include <vector>

#include "bsa_internal.h"

namespace bsa {

struct GatherDesc {
  const void *src;
  void *dst;
  int esz;  // 1, 4 or 8
};
constexpr int kMaxGather = 40;
struct GatherBatch {
  GatherDesc d[kMaxGather];
  int n;
};

// dst[newidx[o]] = src[o] for every kept o (newidx[o] >= 0), all arrays at once
__global__ __launch_bounds__(256) void k_compact(int nold, const int *__restrict__ newidx, GatherBatch b) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= nold) return;
  const int t = newidx[o];
  if (t < 0) return;
  for (int q = 0; q < b.n; ++q) {
    const GatherDesc &g = b.d[q];
    if (g.esz == 8)
      ((unsigned long long *)g.dst)[t] = ((const unsigned long long *)g.src)[o];
    else if (g.esz == 4)
      ((unsigned *)g.dst)[t] = ((const unsigned *)g.src)[o];
    else
      ((uint8_t *)g.dst)[t] = ((const uint8_t *)g.src)[o];
  }
}

struct PerAc {
  DevBuf *b;
  int esz;
  int count;  // sub-arrays of length n in the buffer (the envelope holds 6)
};

// every persistent per-aircraft array of the resident sim
static std::vector<PerAc> per_aircraft(Ctx *c) {
  std::vector<PerAc> v;
  for (int k = 0; k < 6; ++k) v.push_back({&c->own[k], 8, 1});
  DevBuf *f64[] = {&c->s_tas,   &c->s_hdg,   &c->s_gse,    &c->s_gsn,   &c->s_aptrk, &c->s_aptas,
                   &c->s_apalt, &c->s_apvs,  &c->s_selalt, &c->s_bank,  &c->s_eps,   &c->s_accel,
                   &c->s_atrk,  &c->s_atas,  &c->s_avs,    &c->s_aalt,  &c->s_altprev, &c->s_ax,
                   &c->tcpamax};
  for (auto *b : f64) v.push_back({b, 8, 1});
  v.push_back({&c->s_ase, 4, 1});
  v.push_back({&c->s_asn, 4, 1});
  v.push_back({&c->s_active, 1, 1});
  v.push_back({&c->inconf, 1, 1});
  // NORESO / RESOOFF membership and the last ResumeNav's drops (allocated on use)
  for (auto *b : {&c->s_noreso, &c->s_resooff, &c->s_dropped})
    if (b->p) v.push_back({b, 1, 1});
  if (c->sim_limits) v.push_back({&c->s_env, 8, 6});
  if (c->sim_atmos) v.push_back({&c->s_atm, 8, 3});
  if (c->sim_perf) {
    v.push_back({&c->s_ptype, 4, 1});
    v.push_back({&c->s_phase, 1, 1});
  }
  return v;
}

static int check_sim(Ctx *c, const char *what) {
  if (!c->sim_ready) return fail(c, "%s before bsa_sim_init", what);
  if (c->feed_pending) {  // a requested ACDATA snapshot is dropped: its rows are re-laid out
    BSA_HIP(c, hipEventSynchronize(c->feed_ev));
    c->feed_pending = false;
  }
  return 0;
}

// download a CSR (ptr: rows + 1 words, col: ptr[rows] words)
static int get_csr(Ctx *c, const DevBuf &ptr, const DevBuf &col, int64_t rows, std::vector<unsigned> &p,
                   std::vector<unsigned> &q) {
  p.assign((size_t)rows + 1, 0u);
  BSA_HIP(c, hipMemcpyAsync(p.data(), ptr.p, p.size() * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  q.assign(p[(size_t)rows], 0u);
  if (!q.empty()) BSA_HIP(c, hipMemcpyAsync(q.data(), col.p, q.size() * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

static int put_csr(Ctx *c, DevBuf &ptr, DevBuf &col, const std::vector<unsigned> &p,
                   const std::vector<unsigned> &q, size_t colcap, const char *what) {
  if (!ensure_keep(c, ptr, p.size() * 4, what) || !ensure_keep(c, col, std::max(q.size(), colcap) * 4, what))
    return -1;
  BSA_HIP(c, hipMemcpyAsync(ptr.p, p.data(), p.size() * 4, hipMemcpyHostToDevice, c->stream));
  if (!q.empty()) BSA_HIP(c, hipMemcpyAsync(col.p, q.data(), q.size() * 4, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));  // the host vectors go out of scope
  return 0;
}

// rows of CSR (p, q) over homes kept by nh (old home -> new home, -1 = the
// ownship was deleted: its pairs go, asas.py:421-423), columns mapped by nid
// (old index -> new, -1 = deleted intruder: kDangling with `dangling`, else
// dropped); rows appended for created aircraft (empty)
static void remap_csr(const std::vector<unsigned> &p, const std::vector<unsigned> &q, const std::vector<int> &nh,
                      const std::vector<int> &nid, bool dangling, int64_t created, std::vector<unsigned> &np,
                      std::vector<unsigned> &nq) {
  np.assign(1, 0u);
  nq.clear();
  for (size_t o = 0; o + 1 < p.size(); ++o) {
    if (nh[o] < 0) continue;
    bool dang = false;
    for (unsigned e = p[o]; e < p[o + 1]; ++e) {
      const unsigned j = q[e];
      if (j == kDangling || nid[j] < 0)
        dang = true;  // intruder deleted (now or before the last CD call)
      else
        nq.push_back((unsigned)nid[j]);
    }
    if (dang && dangling) nq.push_back(kDangling);  // one marker per row is enough
    np.push_back((unsigned)nq.size());
  }
  for (int64_t k = 0; k < created; ++k) np.push_back((unsigned)nq.size());
}

// ---- several ranks.  Before a delete / create every rank completes its
// replicas (every rank's rows of every per-aircraft array: one all-gather),
// and the ASAS bookkeeping of all ranks (resopairs rows, the previous call's
// gathered pair keys) comes to every rank's host, so the change is the same
// computation everywhere; afterwards the rows are re-partitioned over the new
// n (set_rank_rows) and each rank keeps the bookkeeping of its new range.
struct RowDesc {
  char *p;
  int esz;
};
constexpr int kMaxRowDesc = 32;
struct RowBatch {
  RowDesc d[kMaxRowDesc];
  int n, rowbytes;
};

template <typename T>
__device__ __forceinline__ void cp_row(char *dst, const char *src) {
  *reinterpret_cast<T *>(dst) = *reinterpret_cast<const T *>(src);
}
__device__ __forceinline__ void cp_esz(int esz, char *dst, const char *src) {
  if (esz == 8) cp_row<unsigned long long>(dst, src);
  else if (esz == 4) cp_row<unsigned>(dst, src);
  else *dst = *src;
}

// this rank's rows [rb, re) of every array into its block (array k at rpr x
// (sum of the earlier arrays' element sizes))
__global__ __launch_bounds__(256) void k_rows_pack(int rb, int re, int rpr, RowBatch b, char *__restrict__ send) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rpr || rb + r >= re) return;
  size_t off = 0;
  for (int k = 0; k < b.n; ++k) {
    const int e = b.d[k].esz;
    cp_esz(e, send + off + (size_t)r * e, b.d[k].p + (size_t)(rb + r) * e);
    off += (size_t)rpr * e;
  }
}

__global__ __launch_bounds__(256) void k_rows_unpack(int n, int rpr, int me, RowBatch b, const char *__restrict__ recv) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= n) return;
  const int q = h / rpr, r = h - q * rpr;
  if (q == me) return;
  const char *blk = recv + (size_t)q * rpr * b.rowbytes;
  size_t off = 0;
  for (int k = 0; k < b.n; ++k) {
    const int e = b.d[k].esz;
    cp_esz(e, b.d[k].p + (size_t)h * e, blk + off + (size_t)r * e);
    off += (size_t)rpr * e;
  }
}

static int gather_rows(Ctx *c, const std::vector<PerAc> &arrs) {
  const int64_t n = c->n, rpr = c->sim_rpr;
  std::vector<RowDesc> ds;
  for (const PerAc &pa : arrs) {
    if (!pa.b->p) continue;
    for (int s = 0; s < pa.count; ++s) ds.push_back(RowDesc{(char *)pa.b->p + (size_t)s * n * pa.esz, pa.esz});
  }
  DevBuf snd, rcv;
  struct Rel {
    DevBuf *a, *b;
    ~Rel() {
      release(*a);
      release(*b);
    }
  } rel{&snd, &rcv};
  for (size_t k0 = 0; k0 < ds.size(); k0 += kMaxRowDesc) {
    RowBatch b{};
    for (size_t k = k0; k < ds.size() && b.n < kMaxRowDesc; ++k) {
      b.d[b.n++] = ds[k];
      b.rowbytes += ds[k].esz;
    }
    const size_t blk = (size_t)rpr * b.rowbytes;
    if (!ensure(c, snd, std::max<size_t>(blk, 16), "row gather send") ||
        !ensure(c, rcv, std::max<size_t>(blk * c->nranks, 16), "row gather recv"))
      return -1;
    hipLaunchKernelGGL(k_rows_pack, dim3((unsigned)((rpr + 255) / 256)), dim3(256), 0, c->stream, (int)c->sim_rb,
                       (int)c->sim_re, (int)rpr, b, (char *)snd.p);
    BSA_HIP(c, hipGetLastError());
    if (comm_allgather(c, snd.p, rcv.p, blk)) return -1;
    hipLaunchKernelGGL(k_rows_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n, (int)rpr,
                       c->rank, b, (const char *)rcv.p);
    BSA_HIP(c, hipGetLastError());
  }
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// every rank's vector of words on every rank (host)
static int allgather_words(Ctx *c, const std::vector<unsigned> &mine, std::vector<std::vector<unsigned>> &all) {
  const int R = c->nranks;
  std::vector<double> sz((size_t)R, 0.0);
  sz[(size_t)c->rank] = (double)mine.size();
  if (comm_allreduce_host(c, sz.data(), R, false)) return -1;
  size_t w = 1;
  for (double x : sz) w = std::max(w, (size_t)x);
  DevBuf snd, rcv;
  struct Rel {
    DevBuf *a, *b;
    ~Rel() {
      release(*a);
      release(*b);
    }
  } rel{&snd, &rcv};
  if (!ensure(c, snd, w * 4, "word gather send") || !ensure(c, rcv, w * 4 * R, "word gather recv")) return -1;
  if (!mine.empty())
    BSA_HIP(c, hipMemcpyAsync(snd.p, mine.data(), mine.size() * 4, hipMemcpyHostToDevice, c->stream));
  if (comm_allgather(c, snd.p, rcv.p, w * 4)) return -1;
  std::vector<unsigned> h(w * R);
  BSA_HIP(c, hipMemcpyAsync(h.data(), rcv.p, h.size() * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  all.assign((size_t)R, {});
  for (int q = 0; q < R; ++q) all[(size_t)q].assign(h.begin() + (size_t)q * w, h.begin() + (size_t)q * w + (size_t)sz[(size_t)q]);
  return 0;
}

struct Multi {
  bool on = false;
  DevBuf ginc, gtcp;                      // inconf / tcpamax of the last CD call, full n (home order)
  std::vector<unsigned> gp, gq;           // resopairs of every rank's rows (n home rows)
  std::vector<unsigned long long> keys;   // the previous call's gathered pair-key blocks (R x W)
  ~Multi() {
    release(ginc);
    release(gtcp);
  }
};

// the per-aircraft arrays to carry through the change (several ranks: the
// per-row outputs of the last detect as their full-n copies)
static std::vector<PerAc> change_arrays(Ctx *c, Multi &m) {
  std::vector<PerAc> v = per_aircraft(c);
  if (m.on)
    for (auto &pa : v) {
      if (pa.b == &c->inconf) pa.b = &m.ginc;
      if (pa.b == &c->tcpamax) pa.b = &m.gtcp;
    }
  return v;
}

static int multi_begin(Ctx *c, Multi &m) {
  m.on = c->nranks > 1;
  if (!m.on) return 0;
  const int64_t n = c->n, rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  if (!ensure(c, m.ginc, (size_t)n, "inconf") || !ensure(c, m.gtcp, (size_t)n * 8, "tcpamax")) return -1;
  BSA_HIP(c, hipMemsetAsync(m.ginc.p, 0, (size_t)n, c->stream));
  BSA_HIP(c, hipMemsetAsync(m.gtcp.p, 0, (size_t)n * 8, c->stream));
  if (nr > 0 && c->inconf.p && c->tcpamax.p && c->sim_cd_calls > 0) {
    BSA_HIP(c, hipMemcpyAsync((char *)m.ginc.p + rb, c->inconf.p, (size_t)nr, hipMemcpyDeviceToDevice, c->stream));
    BSA_HIP(c, hipMemcpyAsync((char *)m.gtcp.p + (size_t)rb * 8, c->tcpamax.p, (size_t)nr * 8, hipMemcpyDeviceToDevice,
                              c->stream));
  }
  if (gather_rows(c, change_arrays(c, m))) return -1;
  if (!c->bk_ready) return 0;
  // resopairs: [ptr (rows + 1) | cols] of every rank
  std::vector<unsigned> p, q;
  if (nr > 0) {
    if (get_csr(c, c->bk_rptr, c->bk_rcol, nr, p, q)) return -1;
  } else {
    p.assign(1, 0u);
  }
  std::vector<unsigned> mine = p;
  mine.insert(mine.end(), q.begin(), q.end());
  std::vector<std::vector<unsigned>> all;
  if (allgather_words(c, mine, all)) return -1;
  m.gp.assign(1, 0u);
  m.gq.clear();
  for (int r = 0; r < c->nranks; ++r) {
    const int64_t rrb = std::min<int64_t>(n, (int64_t)r * c->sim_rpr), rre = std::min<int64_t>(n, rrb + c->sim_rpr);
    const std::vector<unsigned> &v = all[(size_t)r];
    const size_t rows = (size_t)(rre - rrb);
    if (v.size() < rows + 1) return fail(c, "resopairs gather: rank %d sent %zu words for %zu rows", r, v.size(), rows);
    const unsigned base = (unsigned)m.gq.size();
    for (size_t k = 1; k <= rows; ++k) m.gp.push_back(base + v[k]);
    m.gq.insert(m.gq.end(), v.begin() + rows + 1, v.begin() + rows + 1 + v[rows]);
  }
  // the previous call's pair keys: the same blocks on every rank
  if (c->bk_kw_alloc) {
    m.keys.assign((size_t)c->bk_kw_alloc * c->nranks, 0ull);
    BSA_HIP(c, hipMemcpyAsync(m.keys.data(), c->bk_kprev.p, m.keys.size() * 8, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
  }
  return 0;
}

// new n: one rank owns everything; several ranks re-partition (512-aligned home ranges)
static void set_n(Ctx *c, int64_t n) {
  c->n = n;
  if (c->nranks > 1) {
    set_rank_rows(c);
  } else {
    c->sim_rpr = n;
    c->sim_rb = 0;
    c->sim_re = n;
  }
  c->last_rb = c->sim_rb;
  c->last_re = c->sim_re;
  c->have_pairs = false;
  c->perm_valid = false;   // the spatial order is over the old indices
  c->reuse_valid = false;  // so is any reusable candidate list
  c->sim_gathered = true;  // every replica is complete after the change
  c->sim_prepped = false;  // prepared records are of the old traffic
  c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
}

// length of each full-n per-aircraft buffer for n aircraft (several ranks: the
// in-place all-gather of the sharded step reaches nranks x rpr rows)
static size_t rows_alloc(const Ctx *c, int64_t n) {
  const int64_t R = c->nranks;
  const int64_t rpr = ((n + R - 1) / R + kTile - 1) / kTile * kTile;
  return (size_t)std::max<int64_t>(n, R > 1 ? R * rpr : n);
}

static int multi_end(Ctx *c, Multi &m, const std::vector<int> &nh, const std::vector<int> &nid, int64_t created) {
  if (!m.on) return 0;
  const int64_t n = c->n, rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  // this rank's rows of the last detect's per-row outputs
  if (!ensure_keep(c, c->inconf, (size_t)std::max<int64_t>(nr, 1), "inconf") ||
      !ensure_keep(c, c->tcpamax, (size_t)std::max<int64_t>(nr, 1) * 8, "tcpamax"))
    return -1;
  if (nr > 0) {
    BSA_HIP(c, hipMemcpyAsync(c->inconf.p, (const char *)m.ginc.p + rb, (size_t)nr, hipMemcpyDeviceToDevice, c->stream));
    BSA_HIP(c, hipMemcpyAsync(c->tcpamax.p, (const char *)m.gtcp.p + (size_t)rb * 8, (size_t)nr * 8,
                              hipMemcpyDeviceToDevice, c->stream));
  }
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  if (c->bk_ready) {
    // resopairs: the global CSR through the change, then this rank's new rows
    std::vector<unsigned> np, nq;
    remap_csr(m.gp, m.gq, nh, nid, true, created, np, nq);
    std::vector<unsigned> p((size_t)nr + 1), q;
    for (int64_t k = 0; k <= nr; ++k) p[(size_t)k] = np[(size_t)(rb + k)] - np[(size_t)rb];
    q.assign(nq.begin() + np[(size_t)rb], nq.begin() + np[(size_t)(rb + nr)]);
    if (put_csr(c, c->bk_rptr, c->bk_rcol, p, q, (size_t)c->bk_cap, "resopairs")) return -1;
    // previous call's pair keys (home row << 32 | index), re-bucketed by the new
    // ranges (a monotone remap keeps the concatenated lists sorted)
    if (!m.keys.empty()) {
      const int R = c->nranks;
      const size_t W0 = (size_t)c->bk_kw_alloc;
      std::vector<std::vector<unsigned long long>> lst[2];
      lst[0].assign((size_t)R, {});
      lst[1].assign((size_t)R, {});
      for (int r = 0; r < R; ++r) {
        const unsigned long long *b = m.keys.data() + (size_t)r * W0;
        const unsigned long long P[2] = {b[0], b[1]};
        const unsigned long long *k = b + 2;
        for (int l = 0; l < 2; ++l) {
          for (unsigned long long x = 0; x < P[l]; ++x) {
            const unsigned long long key = k[(l ? P[0] : 0) + x];
            const unsigned h = (unsigned)(key >> 32), j = (unsigned)key;
            if (h >= nh.size() || j >= nid.size() || nh[h] < 0 || nid[j] < 0) continue;
            const unsigned h2 = (unsigned)nh[h];
            lst[l][(size_t)(h2 / (unsigned)c->sim_rpr)].push_back((unsigned long long)h2 << 32 | (unsigned)nid[j]);
          }
        }
      }
      size_t W = std::max<size_t>((size_t)c->bk_kw, 2);
      for (int r = 0; r < R; ++r) W = std::max(W, 2 + lst[0][(size_t)r].size() + lst[1][(size_t)r].size());
      std::vector<unsigned long long> nb((size_t)R * W, 0ull);
      for (int r = 0; r < R; ++r) {
        unsigned long long *b = nb.data() + (size_t)r * W;
        b[0] = lst[0][(size_t)r].size();
        b[1] = lst[1][(size_t)r].size();
        std::copy(lst[0][(size_t)r].begin(), lst[0][(size_t)r].end(), b + 2);
        std::copy(lst[1][(size_t)r].begin(), lst[1][(size_t)r].end(), b + 2 + b[0]);
      }
      c->bk_kw = c->bk_kw_alloc = W;  // the same on every rank (the same data)
      if (!ensure(c, c->bk_kprev, nb.size() * 8, "previous gathered pair keys")) return -1;
      BSA_HIP(c, hipMemcpyAsync(c->bk_kprev.p, nb.data(), nb.size() * 8, hipMemcpyHostToDevice, c->stream));
      BSA_HIP(c, hipStreamSynchronize(c->stream));
    }
  }
  (void)n;
  // the halo plan's capacities for the new partition (every replica is complete)
  return halo_init_caps(c);
}

}  // namespace bsa

using bsa::Ctx;

extern "C" {

int bsa_sim_delete(bsa_ctx *cc, int64_t k, const int64_t *idx) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (bsa::check_sim(c, "bsa_sim_delete")) return -1;
  if (k < 0 || (k > 0 && !idx)) return bsa::fail(c, "bad delete list");
  const int64_t n = c->n;
  std::vector<int64_t> d(idx, idx + k);
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  if (!d.empty() && (d.front() < 0 || d.back() >= n)) return bsa::fail(c, "delete index out of range [0, %lld)", (long long)n);
  if ((int64_t)d.size() >= n) return bsa::fail(c, "bsa_sim_delete would remove every aircraft: re-init instead");
  if (d.empty()) return 0;
  BSA_HIP(c, hipSetDevice(c->device));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  bsa::Multi mu;
  if (bsa::multi_begin(c, mu)) return -1;
  // old index -> new index (np.delete keeps the order of the rest), -1 = deleted
  std::vector<int> nid((size_t)n);
  {
    size_t q = 0;
    int run = 0;
    for (int64_t o = 0; o < n; ++o) {
      if (q < d.size() && d[q] == o) {
        nid[(size_t)o] = -1;
        ++q;
      } else {
        nid[(size_t)o] = run++;
      }
    }
  }
  const int64_t nn = n - (int64_t)d.size();
  // the arrays are in home order: old home -> new home (the kept homes keep
  // their order), and the new home -> index map
  std::vector<int> nh((size_t)n);
  std::vector<unsigned> h2id_new((size_t)nn);
  {
    int run = 0;
    for (int64_t h = 0; h < n; ++h) {
      const int id = nid[c->h2id_h[(size_t)h]];
      nh[(size_t)h] = id < 0 ? -1 : run;
      if (id >= 0) h2id_new[(size_t)run++] = (unsigned)id;
    }
  }
  bsa::DevBuf map;
  if (!bsa::ensure(c, map, (size_t)n * 4, "delete map")) return -1;
  BSA_HIP(c, hipMemcpyAsync(map.p, nh.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  // gather every per-aircraft array into a fresh buffer, then swap
  std::vector<bsa::PerAc> arrs = bsa::change_arrays(c, mu);
  struct Fresh {  // released unless swapped in (error paths)
    std::vector<bsa::DevBuf> b;
    bsa::DevBuf map;
    ~Fresh() {
      for (auto &x : b) bsa::release(x);
      bsa::release(map);
    }
  } keep;
  std::vector<bsa::DevBuf> &fresh = keep.b;
  fresh.resize(arrs.size());
  keep.map = map;
  map = bsa::DevBuf{};
  const int *dmap = (const int *)keep.map.p;
  bsa::GatherBatch gb{};
  auto launch = [&]() -> int {
    if (!gb.n) return 0;
    hipLaunchKernelGGL(bsa::k_compact, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n, dmap,
                       gb);
    BSA_HIP(c, hipGetLastError());
    gb.n = 0;
    return 0;
  };
  const size_t NA = bsa::rows_alloc(c, nn);
  for (size_t a = 0; a < arrs.size(); ++a) {
    const bsa::PerAc &pa = arrs[a];
    if (!pa.b->p) continue;
    if (!bsa::ensure(c, fresh[a], (pa.count == 1 ? NA : (size_t)nn) * pa.esz * pa.count, "compacted traffic array"))
      return -1;
    for (int s = 0; s < pa.count; ++s) {
      if (gb.n == bsa::kMaxGather && launch()) return -1;
      gb.d[gb.n++] = bsa::GatherDesc{(const char *)pa.b->p + (size_t)s * n * pa.esz,
                                     (char *)fresh[a].p + (size_t)s * nn * pa.esz, pa.esz};
    }
  }
  if (launch()) return -1;
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  for (size_t a = 0; a < arrs.size(); ++a) {
    if (!arrs[a].b->p) continue;
    bsa::release(*arrs[a].b);
    *arrs[a].b = fresh[a];
    fresh[a] = bsa::DevBuf{};
  }
  // ASAS bookkeeping (asas.py:409-504): remap the CSRs of the resopairs and
  // (one rank) of the previous call's conflict / LoS pairs (rows = homes,
  // columns = aircraft indices); several ranks: multi_end
  if (c->bk_ready && !mu.on) {
    std::vector<unsigned> p, q, np, nq;
    auto remap = [&](bsa::DevBuf &ptr, bsa::DevBuf &col, bool dangling, size_t colcap, const char *what) -> int {
      if (bsa::get_csr(c, ptr, col, n, p, q)) return -1;
      bsa::remap_csr(p, q, nh, nid, dangling, 0, np, nq);
      return bsa::put_csr(c, ptr, col, np, nq, colcap, what);
    };
    if (remap(c->bk_rptr, c->bk_rcol, true, (size_t)c->bk_cap, "resopairs") ||
        remap(c->bk_pcptr, c->bk_pccol, false, (size_t)c->cand_cap, "previous conflicts") ||
        remap(c->bk_plptr, c->bk_plcol, false, (size_t)std::max(c->cand_cap, c->los_cap), "previous los"))
      return -1;
  }
  bsa::set_n(c, nn);
  c->h2id_h = h2id_new;
  if (bsa::set_home_maps(c)) return -1;
  return bsa::multi_end(c, mu, nh, nid, 0);
}

int bsa_sim_create(bsa_ctx *cc, int64_t m, const bsa_sim_state *s) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (bsa::check_sim(c, "bsa_sim_create")) return -1;
  if (m < 1 || !s) return bsa::fail(c, "bad create arguments");
  if (c->sim_limits || c->sim_perf)
    return bsa::fail(c, "bsa_sim_create with OpenAP limits on: switch them off, create, set them again");
  const double *src[] = {s->lat, s->lon, s->alt, s->tas, s->hdg, s->vs, s->gs, s->trk, s->gseast,
                         s->gsnorth, s->ap_trk, s->ap_tas, s->ap_alt, s->ap_vs, s->selalt, s->bank,
                         s->eps, s->accel, s->asas_alt};
  for (auto q : src)
    if (!q) return bsa::fail(c, "bsa_sim_create: NULL array");
  const int64_t n = c->n, nn = n + m;
  if (nn > 0x7fffffff) return bsa::fail(c, "n would exceed 2^31-1");
  BSA_HIP(c, hipSetDevice(c->device));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  bsa::Multi mu;
  if (bsa::multi_begin(c, mu)) return -1;
  std::vector<bsa::PerAc> arrs = bsa::change_arrays(c, mu);
  const size_t NA = bsa::rows_alloc(c, nn);
  for (auto &pa : arrs)
    if (!bsa::ensure_keep(c, *pa.b, (pa.count == 1 ? NA : (size_t)nn) * pa.esz * pa.count, "traffic array"))
      return -1;
  const size_t M8 = (size_t)m * 8;
  struct {
    bsa::DevBuf *b;
    const double *h;
  } put[] = {{&c->own[0], s->lat},      {&c->own[1], s->lon},      {&c->own[2], s->trk},
             {&c->own[3], s->gs},       {&c->own[4], s->alt},      {&c->own[5], s->vs},
             {&c->s_tas, s->tas},       {&c->s_hdg, s->hdg},       {&c->s_gse, s->gseast},
             {&c->s_gsn, s->gsnorth},   {&c->s_aptrk, s->ap_trk},  {&c->s_aptas, s->ap_tas},
             {&c->s_apalt, s->ap_alt},  {&c->s_apvs, s->ap_vs},    {&c->s_selalt, s->selalt},
             {&c->s_bank, s->bank},     {&c->s_eps, s->eps},       {&c->s_accel, s->accel},
             {&c->s_atrk, s->trk},      {&c->s_atas, s->tas},      {&c->s_aalt, s->asas_alt},  // asas.py:402-407
             {&c->s_altprev, s->alt}};
  for (auto &e : put)
    BSA_HIP(c, hipMemcpyAsync((char *)e.b->p + (size_t)n * 8, e.h, M8, hipMemcpyHostToDevice, c->stream));
  // defaults of TrafficArrays.create (trafficarrays.py:73-95): 0 / False
  struct {
    bsa::DevBuf *b;
    int esz;
  } zero[] = {{&c->s_avs, 8}, {&c->s_ax, 8}, {mu.on ? &mu.gtcp : &c->tcpamax, 8}, {&c->s_ase, 4}, {&c->s_asn, 4},
              {&c->s_active, 1}, {mu.on ? &mu.ginc : &c->inconf, 1}};
  for (auto &z : zero)
    BSA_HIP(c, hipMemsetAsync((char *)z.b->p + (size_t)n * z.esz, 0, (size_t)m * z.esz, c->stream));
  for (auto *b : {&c->s_noreso, &c->s_resooff, &c->s_dropped})  // not in the lists, nothing dropped
    if (b->p) BSA_HIP(c, hipMemsetAsync((char *)b->p + n, 0, (size_t)m, c->stream));
  if (c->sim_atmos) {  // the atmosphere's three sub-arrays move to the new stride n + m (via a copy:
    bsa::DevBuf tmp;    // the old and new places of a sub-array may overlap)
    if (!bsa::ensure(c, tmp, (size_t)n * 24, "atmosphere")) return -1;
    BSA_HIP(c, hipMemcpyAsync(tmp.p, c->s_atm.p, (size_t)n * 24, hipMemcpyDeviceToDevice, c->stream));
    BSA_HIP(c, hipMemsetAsync(c->s_atm.p, 0, (size_t)nn * 24, c->stream));
    for (int k = 0; k < 3; ++k)
      BSA_HIP(c, hipMemcpyAsync((char *)c->s_atm.p + (size_t)k * nn * 8, (char *)tmp.p + (size_t)k * n * 8,
                                (size_t)n * 8, hipMemcpyDeviceToDevice, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    bsa::release(tmp);
  }
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  // new aircraft have no resopairs and were in no previous pair set: empty CSR rows
  std::vector<int> ident((size_t)n);
  for (int64_t k = 0; k < n; ++k) ident[(size_t)k] = (int)k;
  if (c->bk_ready && !mu.on) {
    std::vector<unsigned> p, q;
    bsa::DevBuf *csr[3][2] = {{&c->bk_rptr, &c->bk_rcol}, {&c->bk_pcptr, &c->bk_pccol}, {&c->bk_plptr, &c->bk_plcol}};
    const size_t caps[3] = {(size_t)c->bk_cap, (size_t)c->cand_cap, (size_t)std::max(c->cand_cap, c->los_cap)};
    for (int k = 0; k < 3; ++k) {
      if (bsa::get_csr(c, *csr[k][0], *csr[k][1], n, p, q)) return -1;
      p.resize((size_t)nn + 1, p.back());
      if (bsa::put_csr(c, *csr[k][0], *csr[k][1], p, q, caps[k], "bookkeeping rows")) return -1;
    }
  }
  bsa::set_n(c, nn);
  // the new aircraft's gseast / gsnorth are the host's (numpy's sin / cos), not
  // K4's expressions of their gs / trk: the halo sends them until K4' has run
  c->sim_gs_derivable = false;
  // the new aircraft take the homes after the existing ones, in index order
  for (int64_t k = n; k < nn; ++k) c->h2id_h.push_back((unsigned)k);
  if (bsa::set_home_maps(c)) return -1;
  return bsa::multi_end(c, mu, ident, ident, m);
}

}  // extern "C"
