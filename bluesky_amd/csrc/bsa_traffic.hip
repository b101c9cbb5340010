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
// One rank only: with several ranks the row partition would move rows (and
// their bookkeeping) between GPUs; re-init the sim there.
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
  if (c->nranks > 1) return fail(c, "%s with several ranks: re-init the sim (rows would move between GPUs)", what);
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

// new sizes after a change of n (one rank: all rows are this rank's)
static void set_n(Ctx *c, int64_t n) {
  c->n = n;
  c->sim_rpr = n;
  c->sim_rb = 0;
  c->sim_re = n;
  c->last_rb = 0;
  c->last_re = n;
  c->have_pairs = false;
  c->perm_valid = false;   // the spatial order is over the old indices
  c->reuse_valid = false;  // so is any reusable candidate list
  c->sim_gathered = true;
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
  std::vector<bsa::PerAc> arrs = bsa::per_aircraft(c);
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
  for (size_t a = 0; a < arrs.size(); ++a) {
    const bsa::PerAc &pa = arrs[a];
    if (!pa.b->p) continue;
    if (!bsa::ensure(c, fresh[a], (size_t)nn * pa.esz * pa.count, "compacted traffic array")) return -1;
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
  // of the previous call's conflict / LoS pairs (rows = all n homes on one
  // rank, columns = aircraft indices)
  if (c->bk_ready) {
    std::vector<unsigned> p, q, np, nq;
    auto remap = [&](bsa::DevBuf &ptr, bsa::DevBuf &col, bool dangling, size_t colcap, const char *what) -> int {
      if (bsa::get_csr(c, ptr, col, n, p, q)) return -1;
      np.assign(1, 0u);
      nq.clear();
      for (int64_t o = 0; o < n; ++o) {
        if (nh[(size_t)o] < 0) continue;  // ownship deleted: its pairs go (asas.py:421-423)
        bool dang = false;
        for (unsigned e = p[(size_t)o]; e < p[(size_t)o + 1]; ++e) {
          const unsigned j = q[e];
          if (j == bsa::kDangling || nid[j] < 0) {
            dang = true;  // intruder deleted
          } else {
            nq.push_back((unsigned)nid[j]);
          }
        }
        if (dang && dangling) nq.push_back(bsa::kDangling);  // one marker per row is enough
        np.push_back((unsigned)nq.size());
      }
      return bsa::put_csr(c, ptr, col, np, nq, colcap, what);
    };
    if (remap(c->bk_rptr, c->bk_rcol, true, (size_t)c->bk_cap, "resopairs") ||
        remap(c->bk_pcptr, c->bk_pccol, false, (size_t)c->cand_cap, "previous conflicts") ||
        remap(c->bk_plptr, c->bk_plcol, false, (size_t)std::max(c->cand_cap, c->los_cap), "previous los"))
      return -1;
  }
  bsa::set_n(c, nn);
  c->h2id_h = h2id_new;
  return bsa::set_home_maps(c);
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
  std::vector<bsa::PerAc> arrs = bsa::per_aircraft(c);
  for (auto &pa : arrs)
    if (!bsa::ensure_keep(c, *pa.b, (size_t)nn * pa.esz, "traffic array")) return -1;
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
  } zero[] = {{&c->s_avs, 8}, {&c->s_ax, 8}, {&c->tcpamax, 8}, {&c->s_ase, 4}, {&c->s_asn, 4},
              {&c->s_active, 1}, {&c->inconf, 1}};
  for (auto &z : zero)
    BSA_HIP(c, hipMemsetAsync((char *)z.b->p + (size_t)n * z.esz, 0, (size_t)m * z.esz, c->stream));
  for (auto *b : {&c->s_noreso, &c->s_resooff, &c->s_dropped})  // not in the lists, nothing dropped
    if (b->p) BSA_HIP(c, hipMemsetAsync((char *)b->p + n, 0, (size_t)m, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  // new aircraft have no resopairs and were in no previous pair set: empty CSR rows
  if (c->bk_ready) {
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
  // the new aircraft take the homes after the existing ones, in index order
  for (int64_t k = n; k < nn; ++k) c->h2id_h.push_back((unsigned)k);
  return bsa::set_home_maps(c);
}

}  // extern "C"
