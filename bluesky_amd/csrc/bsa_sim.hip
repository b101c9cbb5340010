// GPU-resident sim step and the RCCL row-sharded multi-GPU mode.
//
// One step, rows [rb, re) owned by this rank:
//   every cd_every steps:
//     C1  all-gather of the 8 state arrays CD/MVP read for other rows
//         (lat lon trk gs alt vs gseast gsnorth) over xGMI, one RCCL call
//     K0-K2 detect(own rows x all columns)          asas.py:481-483
//     C2  all-reduce(max) of the 2-word gate {candidate overflow, P} (RCCL,
//         device buffer; skipped on one rank)
//     K3  MVP on the own rows' pairs, only when some rank has a conflict
//         (asas.py:486-487 `if self.confpairs`), and asas.active = inconf
//   every step:
//     K4' Pilot.APorASAS (no wind, pilot.py:41-63) fused with the kinematic
//         update (traffic.py:425-483) of the own rows
//
// A batch of steps is enqueued without any host synchronisation; the gate is
// read on the device.  A candidate-list overflow sets a sticky abort flag:
// every later kernel that writes persistent state (K3, K4') becomes a no-op,
// so the state stays exactly as before the failed step; the host then grows
// the buffers and re-runs the batch from that step.
#include <algorithm>
#include <type_traits>

#include "bsa_kin_math.h"
#include "bsa_mvp_row.h"
#include "bsa_prep.h"
#include "bsa_sim_row.h"

#pragma clang fp contract(off)

namespace bsa {

// Pilot.APorASAS (pilot.py:28-63; no wind, constant wind or a 2-D field) +
// UpdateAirSpeed/GroundSpeed/Position, rows [rb, re).  FUSE (a CD step without
// the ASAS bookkeeping): K3's per-row part (bsa_mvp_row.h: the dv fold, the
// finalize, asas.active = inconf, or DoNothing) runs first in the same lane --
// the row's new ASAS targets are what its pilot reads next (traffic.py:397),
// one launch and one pass over the row state fewer.  The gate check of
// k_mvp_row is made by every lane, so the whole grid agrees on an abort.
// PREP (one rank, the next step is a CD step): the lane also writes the next
// detect's column record of its row from the state it has just computed
// (bsa_prep.h: k_prep_cols' expressions, bitwise its records), and each wave
// reduces its group's sub-group and group boxes; that detect then skips its
// K0b launch, its K0z unites the group boxes into tile boxes
// (detect_enqueue, Ctx::sim_prepped).
template <bool FUSE, bool PREP>
__global__ __launch_bounds__(256) void k_sim_pilot_kin(int rb, int re, double simdt, int winddim, double vwn,
                                                         double vwe, WindField wf, SimDev d, MvpIn mv,
                                                         bsa_mvp_params mp, PrepArgs pa, HkPub pub) {
  const bool stop = *d.sticky != 0u || (FUSE && mv.gate[0] >= kGateOverflow);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (FUSE && mv.gate[0] >= kGateOverflow) mv.sticky[0] = 1u;
    hk_publish(pub, [&] { return stop; });  // HK: the CD step's prediction to the host (also when it aborts)
  }
  if (stop) return;
  const int k = rb + blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) *d.steps_done += 1;
  if (PREP) {  // every lane reaches the wave's group reduction (its record from registers)
    PFRec p{}, b{};
    if (pa.snap && k < re) b = pa.snap[k];  // (issued with the row's other loads)
    if (k < re) p = pilot_kin_row<FUSE, PREP>(rb, k, simdt, winddim, vwn, vwe, wf, d, mv, mp, pa);
    group_boxes_v(pa.n, k / kGroup, p, pa.sbox, pa.gbox);
    if (pa.snap) {
      const bool out = k < re && !pf_within(p, b, pa.dx, pa.ds, pa.dv);
      if (__ballot(out) && (threadIdx.x & 63) == 0) pa.tpr_ctl[0] = 1ull;
      if (pa.pred) {  // HK: ... or pf x the budgets (a rebuild two detects on)
        const bool near = k < re && !pf_within(p, b, pa.pf * pa.dx, pa.pf * pa.ds, pa.pf * pa.dv);
        if (__ballot(near) && (threadIdx.x & 63) == 0) *pa.pred = 1ull;
      }
    }
    return;
  }
  if (k >= re) return;
  pilot_kin_row<FUSE, PREP>(rb, k, simdt, winddim, vwn, vwe, wf, d, mv, mp, pa);
}


// field list of one all-gather: fp64 arrays (full n) + optionally one uint8 array
struct Fields {
  double *f[8];
  int nf;
  uint8_t *u8;  // transported as 0.0 / 1.0 in one extra slot (may be NULL)
};

__global__ __launch_bounds__(256) void k_pack(int rb, int re, int rpr, Fields fl, double *__restrict__ send) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rpr) return;
  const int k = rb + r;
  const bool v = k < re;
  for (int f = 0; f < fl.nf; ++f) send[(size_t)f * rpr + r] = v ? fl.f[f][k] : 0.0;
  if (fl.u8) send[(size_t)fl.nf * rpr + r] = v ? (double)fl.u8[k] : 0.0;
}

__global__ __launch_bounds__(256) void k_unpack(int n, int rpr, int self, Fields fl, int slots,
                                                const double *__restrict__ recv) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int q = k / rpr, r = k - q * rpr;
  if (q == self) return;
  const double *blk = recv + (size_t)q * slots * rpr;
  for (int f = 0; f < fl.nf; ++f) fl.f[f][k] = blk[(size_t)f * rpr + r];
  if (fl.u8) fl.u8[k] = blk[(size_t)fl.nf * rpr + r] != 0.0;
}

static SimDev sim_dev(Ctx *c) {
  SimDev d;
  d.lat = (double *)c->own[0].p;
  d.lon = (double *)c->own[1].p;
  d.trk = (double *)c->own[2].p;
  d.gs = (double *)c->own[3].p;
  d.alt = (double *)c->own[4].p;
  d.vs = (double *)c->own[5].p;
  d.tas = (double *)c->s_tas.p;
  d.hdg = (double *)c->s_hdg.p;
  d.gse = (double *)c->s_gse.p;
  d.gsn = (double *)c->s_gsn.p;
  d.alt_w = d.alt;
  d.vs_w = d.vs;
  d.gse_w = d.gse;
  d.gsn_w = d.gsn;
  d.altprev = (double *)c->s_altprev.p;
  d.ax = (double *)c->s_ax.p;
  d.env = c->sim_limits ? (const double *)c->s_env.p : nullptr;
  d.ptab = c->sim_perf ? (const double *)c->s_ptab.p : nullptr;
  d.ptype = (const int *)c->s_ptype.p;
  d.phase = (uint8_t *)c->s_phase.p;
  d.atm = c->sim_atmos ? (double *)c->s_atm.p : nullptr;
  d.n = (int)c->n;
  d.aptrk = (const double *)c->s_aptrk.p;
  d.aptas = (const double *)c->s_aptas.p;
  d.apalt = (const double *)c->s_apalt.p;
  d.apvs = (const double *)c->s_apvs.p;
  d.bank = (const double *)c->s_bank.p;
  d.eps = (const double *)c->s_eps.p;
  d.accel = (const double *)c->s_accel.p;
  d.atrk = (const double *)c->s_atrk.p;
  d.atas = (const double *)c->s_atas.p;
  d.avs = (const double *)c->s_avs.p;
  d.aalt = (const double *)c->s_aalt.p;
  d.active = (const uint8_t *)c->s_active.p;
  d.sticky = (const unsigned *)((char *)c->sim_ctl.p + bsa::kSimCtlSticky);
  d.steps_done = (unsigned long long *)((char *)c->sim_ctl.p + kSimCtlSteps);
  return d;
}

// one all-gather (RCCL or in-process group) of the listed arrays' rows [sim_rb, sim_re) of every rank
static int gather_fields(Ctx *c, const Fields &fl) {
  const int64_t rpr = c->sim_rpr, n = c->n;
  const int slots = fl.nf + (fl.u8 ? 1 : 0);
  const size_t blk = (size_t)slots * rpr;
  if (!ensure(c, c->g_send, blk * 8, "gather send") ||
      !ensure(c, c->g_recv, blk * 8 * c->nranks, "gather recv"))
    return -1;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((rpr + 255) / 256)), dim3(256), 0, c->stream, (int)c->sim_rb,
                     (int)c->sim_re, (int)rpr, fl, (double *)c->g_send.p);
  BSA_HIP(c, hipGetLastError());
  if (comm_allgather(c, c->g_send.p, c->g_recv.p, blk * 8)) return -1;
  hipLaunchKernelGGL(k_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n,
                     (int)rpr, c->rank, fl, slots, (const double *)c->g_recv.p);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

// Without wind, K4' sets gs = tas, trk = hdg and gseast / gsnorth =
// tas sin / cos(hdg) (traffic.py:455-460, bsa_kin_math.h): every rank derives
// the other ranks' gseast / gsnorth from their gathered gs / trk with the same
// expressions, bitwise, instead of receiving them (6 arrays over xGMI, not 8)
__global__ __launch_bounds__(256) void k_derive_gs(int n, int rb, int re, const double *__restrict__ gs,
                                                   const double *__restrict__ trk, double *__restrict__ gse,
                                                   double *__restrict__ gsn) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n || (k >= rb && k < re)) return;
  double st, ct;
  sincos(trk[k] * kD2R, &st, &ct);  // (as K4''s sincos of hdg)
  gsn[k] = gs[k] * ct;
  gse[k] = gs[k] * st;
}

// C1: replicate every rank's rows of the 8 arrays CD and MVP read for any row
static int sim_gather(Ctx *c) {
  if (c->nranks == 1 || c->sim_gathered) {
    c->sim_gathered = true;
    return 0;
  }
  SimDev d = sim_dev(c);
  // in place: the home ranges are contiguous and the arrays padded to nranks x rpr;
  // gseast / gsnorth are derived when every rank's came from K4' without wind
  double *const f[8] = {d.lat, d.lon, d.trk, d.gs, d.alt, d.vs, d.gse, d.gsn};
  const bool derive = c->simp.winddim == 0 && c->sim_gs_derivable;
  if (comm_allgather_inplace(c, f, derive ? 6 : 8, (size_t)c->sim_rpr)) return -1;
  if (derive) {
    hipLaunchKernelGGL(k_derive_gs, dim3((unsigned)((c->n + 255) / 256)), dim3(256), 0, c->stream, (int)c->n,
                       (int)c->sim_rb, (int)c->sim_re, (const double *)d.gs, (const double *)d.trk, d.gse, d.gsn);
    BSA_HIP(c, hipGetLastError());
  }
  c->sim_gathered = true;
  return 0;
}

// read-time gather of the per-rank ASAS outputs (only own rows are computed)
static int sim_gather_asas(Ctx *c) {
  if (c->nranks == 1) return 0;
  Fields fl{{(double *)c->s_atrk.p, (double *)c->s_atas.p, (double *)c->s_avs.p, (double *)c->s_aalt.p,
             (double *)c->s_tas.p, (double *)c->s_hdg.p, nullptr, nullptr},
            6, (uint8_t *)c->s_active.p};
  return gather_fields(c, fl);
}

// the resident step's last CD call as "the last detect" (its counts are
// read from the device; the host never synchronised on that detect)
int sim_adopt_pairs(Ctx *c) {
  if (c->have_pairs || !c->sim_ready || c->sim_cd_calls == 0) return 0;
  if (c->empty_detect) {
    c->last_conf = c->last_los = 0;
    c->have_pairs = true;
    return 0;
  }
  Counters h;
  BSA_HIP(c, hipMemcpyAsync(&h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  c->last_conf = (int64_t)h.conf;
  c->last_los = (int64_t)h.los;
  c->have_pairs = true;
  return 0;
}

void sim_release(Ctx *c) {
  DevBuf *all[] = {&c->red, &c->s_tas, &c->s_hdg, &c->s_gse, &c->s_gsn, &c->s_aptrk, &c->s_aptas,
                   &c->s_apalt, &c->s_apvs, &c->s_selalt, &c->s_bank, &c->s_eps, &c->s_accel,
                   &c->s_atrk, &c->s_atas, &c->s_avs, &c->s_aalt, &c->s_ase, &c->s_asn,
                   &c->s_active, &c->g_send, &c->g_recv, &c->pg_send, &c->pg_recv, &c->sim_ctl, &c->s_altprev, &c->s_ax, &c->s_env,
                   &c->s_ptab, &c->s_ptype, &c->s_phase, &c->s_noreso, &c->s_resooff, &c->s_dropped, &c->s_atm,
                   &c->xfer_stage, &c->lbyidx, &c->fetch_stage, &c->tpr_snap, &c->tpr_ctl, &c->nx_alt, &c->nx_vs, &c->nx_gse, &c->nx_gsn};
  for (auto *b : all) release(*b);
  bk_release(c);
  halo_release(c);
  comm_release(c);
}

// ---- home order (host side): arrays cross the ABI in aircraft-index order
// and live on the device in home order (Ctx::h2id_h)
template <typename F>
static void by_size(size_t esz, F f) {
  if (esz == 8) f((const uint64_t *)nullptr);
  else if (esz == 4) f((const uint32_t *)nullptr);
  else f((const uint8_t *)nullptr);
}

// Batched home-order transfers of whole arrays (h in [0, n)): the host
// arrays cross PCIe as they are, in aircraft-index order (one async copy
// each into a device staging area), and ONE kernel permutes every field on
// the device -- dst[h] = stage[h2id[h]] on upload, stage[h2id[h]] = src[h] on
// download -- with one stream synchronisation per batch.  (Per array, the
// host-side permutation loop and a synchronisation each cost the ASAS drop-in
// ~0.2 ms per array at 100k aircraft.)
constexpr int kXferMax = 24;
struct XferFields {
  void *dev[kXferMax];
  unsigned long long off[kXferMax];  // byte offset of the field in the staging area
  int esz[kXferMax];
  int nf, up;
};
__global__ __launch_bounds__(256) void k_home_xfer(int n, XferFields f, const unsigned *__restrict__ h2id,
                                                   unsigned char *__restrict__ stage) {
  const int h = blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= n) return;
  const unsigned i = h2id[h];
  for (int q = 0; q < f.nf; ++q) {
    unsigned char *sp = stage + f.off[q];
    unsigned char *dp = (unsigned char *)f.dev[q];
    if (f.esz[q] == 8) {
      if (f.up) ((unsigned long long *)dp)[h] = ((const unsigned long long *)sp)[i];
      else ((unsigned long long *)sp)[i] = ((const unsigned long long *)dp)[h];
    } else if (f.esz[q] == 4) {
      if (f.up) ((unsigned *)dp)[h] = ((const unsigned *)sp)[i];
      else ((unsigned *)sp)[i] = ((const unsigned *)dp)[h];
    } else {
      if (f.up) dp[h] = sp[i];
      else sp[i] = dp[h];
    }
  }
}

struct HomeBatch {
  Ctx *c;
  bool up;
  XferFields f{};
  const void *hsrc[kXferMax] = {};
  void *hdst[kXferMax] = {};
  size_t bytes = 0;
  HomeBatch(Ctx *cc, bool upload) : c(cc), up(upload) { f.up = upload ? 1 : 0; }
  // upload: device array dev <- host src (index order); download: host dst <- dev
  int add(void *dev, const void *hsrc_, void *hdst_, int esz) {
    if (f.nf == kXferMax && run()) return -1;
    const int q = f.nf++;
    f.dev[q] = dev;
    f.esz[q] = esz;
    f.off[q] = bytes;
    hsrc[q] = hsrc_;
    hdst[q] = hdst_;
    bytes += ((size_t)c->n * esz + 255) / 256 * 256;
    return 0;
  }
  int run() {
    const int64_t n = c->n;
    if (f.nf == 0 || n <= 0) return 0;
    if (!ensure(c, c->xfer_stage, bytes, "transfer staging")) return -1;
    unsigned char *st = (unsigned char *)c->xfer_stage.p;
    // the host side through the pinned staging: one parallel host copy and
    // ONE DMA of the whole batch (pin_stage, bsa_ctx.hip)
    unsigned char *pin = pin_stage(c, bytes);
    if (!pin) return -1;
    HostCopy jobs[kXferMax];
    if (up) {
      for (int q = 0; q < f.nf; ++q) jobs[q] = HostCopy{pin + f.off[q], hsrc[q], (size_t)n * f.esz[q]};
      host_copy(jobs, f.nf);
      BSA_HIP(c, hipMemcpyAsync(st, pin, bytes, hipMemcpyHostToDevice, c->stream));
    }
    hipLaunchKernelGGL(k_home_xfer, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n, f,
                       (const unsigned *)c->h2id.p, st);
    BSA_HIP(c, hipGetLastError());
    if (!up) BSA_HIP(c, hipMemcpyAsync(pin, st, bytes, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    if (!up) {
      for (int q = 0; q < f.nf; ++q) jobs[q] = HostCopy{hdst[q], pin + f.off[q], (size_t)n * f.esz[q]};
      host_copy(jobs, f.nf);
    }
    f.nf = 0;
    bytes = 0;
    return 0;
  }
};

// dst[h] (device) = src[h2id[h]] (host), h in [0, n)
static int put_home(Ctx *c, void *dst, const void *src, size_t esz, std::vector<char> &tmp) {
  const int64_t n = c->n;
  tmp.resize((size_t)n * esz + 8);
  const unsigned *H = c->h2id_h.data();
  by_size(esz, [&](auto tag) {
    using T = std::remove_const_t<std::remove_pointer_t<decltype(tag)>>;
    T *t = (T *)tmp.data();
    const T *q = (const T *)src;
    for (int64_t h = 0; h < n; ++h) t[h] = q[H[h]];
  });
  BSA_HIP(c, hipMemcpyAsync(dst, tmp.data(), (size_t)n * esz, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// out[h2id[h]] (host) = src[h] (device), h in [hb, he)
static int get_home(Ctx *c, void *out, const void *src, size_t esz, int64_t hb, int64_t he,
                    std::vector<char> &tmp) {
  if (he <= hb) return 0;
  tmp.resize((size_t)(he - hb) * esz + 8);
  BSA_HIP(c, hipMemcpyAsync(tmp.data(), (const char *)src + (size_t)hb * esz, (size_t)(he - hb) * esz,
                            hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  const unsigned *H = c->h2id_h.data();
  by_size(esz, [&](auto tag) {
    using T = std::remove_const_t<std::remove_pointer_t<decltype(tag)>>;
    const T *t = (const T *)tmp.data();
    T *o = (T *)out;
    for (int64_t h = hb; h < he; ++h) o[H[h]] = t[h - hb];
  });
  return 0;
}

// the maps of a home order h2id_h (host + device) and this rank's lpos
int set_home_maps(Ctx *c) {
  const int64_t n = c->n;
  c->id2h_h.assign((size_t)n, 0u);
  for (int64_t h = 0; h < n; ++h) c->id2h_h[c->h2id_h[(size_t)h]] = (unsigned)h;
  const int64_t rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  std::vector<unsigned> ord((size_t)nr);
  for (int64_t r = 0; r < nr; ++r) ord[(size_t)r] = (unsigned)r;
  std::sort(ord.begin(), ord.end(), [&](unsigned a, unsigned b) { return c->h2id_h[rb + a] < c->h2id_h[rb + b]; });
  c->lpos_h.assign((size_t)nr, 0u);
  for (int64_t k = 0; k < nr; ++k) c->lpos_h[ord[(size_t)k]] = (unsigned)k;
  if (!ensure(c, c->lbyidx, (size_t)std::max<int64_t>(nr, 1) * 4, "rows by index")) return -1;
  if (nr) BSA_HIP(c, hipMemcpyAsync(c->lbyidx.p, ord.data(), (size_t)nr * 4, hipMemcpyHostToDevice, c->stream));
  if (!ensure(c, c->h2id, (size_t)n * 4, "home -> index") || !ensure(c, c->id2h, (size_t)n * 4, "index -> home"))
    return -1;
  BSA_HIP(c, hipMemcpyAsync(c->h2id.p, c->h2id_h.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipMemcpyAsync(c->id2h.p, c->id2h_h.data(), (size_t)n * 4, hipMemcpyHostToDevice, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// rows of `rank`: a 512-aligned home range (the detect's row tiles are then
// column tiles)
void set_rank_rows(Ctx *c) {
  const int64_t n = c->n, R = c->nranks;
  c->sim_rpr = ((n + R - 1) / R + kTile - 1) / kTile * kTile;
  c->sim_rb = std::min<int64_t>(n, (int64_t)c->rank * c->sim_rpr);
  c->sim_re = std::min<int64_t>(n, c->sim_rb + c->sim_rpr);
}

// one CD step of the batch (enqueue only).  allow_defer: K3's per-row part may
// run inside the step's K4' (k_sim_pilot_kin<true>); a CD call without
// kinematics (bsa_sim_cd) launches it itself.
static int sim_cd(Ctx *c, bool allow_defer) {
  const bsa_sim_params &p = c->simp;
  // several ranks: the detect's halo exchange (bsa_halo.hip) refreshes the
  // other ranks' rows this rank reads; one rank holds everything
  if (c->halo_mode != 1 && sim_gather(c)) return -1;
  unsigned long long *gate = (unsigned long long *)c->sim_ctl.p;
  const uint8_t *noreso = c->sim_noreso ? (const uint8_t *)c->s_noreso.p : nullptr;
  const uint8_t *resooff = c->sim_resooff ? (const uint8_t *)c->s_resooff.p : nullptr;
  // MVP's per-pair vectors are evaluated by K2 as it places each pair;
  // k_mvp_row folds them after the gate
  if (p.reso) {
    c->fuse_mvp = &p.mvp;
    c->fuse_gse = (const double *)c->s_gse.p;
    c->fuse_gsn = (const double *)c->s_gsn.p;
    c->fuse_vs = (const double *)c->own[5].p;
    c->fuse_alt = (const double *)c->own[4].p;
    c->fuse_noreso = noreso;
  }
  c->det_home = true;
  const int de = detect_enqueue(c, p.rpz, p.hpz, p.tla, 0, c->sim_rb, c->sim_re, gate);
  c->det_home = false;
  c->fuse_mvp = nullptr;
  c->fuse_noreso = nullptr;
  if (de) return -1;
  c->sim_cd_calls++;
  unsigned *sticky = (unsigned *)((char *)c->sim_ctl.p + bsa::kSimCtlSticky);
  BkDev bk;
  bk.lat = (const double *)c->own[0].p;
  bk.lon = (const double *)c->own[1].p;
  bk.gse = (const double *)c->s_gse.p;
  bk.gsn = (const double *)c->s_gsn.p;
  bk.trk = (const double *)c->own[2].p;
  bk.h2id = (const unsigned *)c->h2id.p;
  bk.id2h = (const unsigned *)c->id2h.p;
  bk.active = (uint8_t *)c->s_active.p;
  bk.dropped = (uint8_t *)c->s_dropped.p;
  bk.gate = gate;
  bk.sticky = sticky;
  bk.demand = (unsigned long long *)((char *)c->sim_ctl.p + kSimCtlDemand);
  bk.kdemand = (unsigned long long *)((char *)c->sim_ctl.p + kSimCtlKdemand);
  // ASAS bookkeeping, first half: kept-pair counts (may flag a resopairs overflow in the gate)
  if (p.resume_nav && bk_count(c, bk)) return -1;
  if (comm_allreduce_max_u64(c, gate, kGateWords)) return -1;
  const int64_t rb = c->sim_rb;
  MvpDev d;
  d.gseast = (const double *)c->s_gse.p;
  d.gsnorth = (const double *)c->s_gsn.p;
  d.vs = (const double *)c->own[5].p;
  d.alt = (const double *)c->own[4].p;
  d.trk = (const double *)c->own[2].p;
  d.gs = (const double *)c->own[3].p;
  d.selalt = (const double *)c->s_selalt.p;
  d.apvs = (const double *)c->s_apvs.p;
  d.aptrk = (const double *)c->s_aptrk.p;
  d.aptas = (const double *)c->s_aptas.p;
  d.apalt = (const double *)c->s_apalt.p;
  d.noreso = noreso;
  d.resooff = resooff;
  d.asas_alt = (double *)c->s_aalt.p + rb;
  d.o_trk = (double *)c->s_atrk.p + rb;
  d.o_tas = (double *)c->s_atas.p + rb;
  d.o_vs = (double *)c->s_avs.p + rb;
  d.o_asase = (float *)c->s_ase.p + rb;
  d.o_asasn = (float *)c->s_asn.p + rb;
  d.o_tsolv = nullptr;
  // K3 (+ gate, + asas.active = inconf unless ResumeNav runs) on the detect's own row offsets
  // without the bookkeeping (which runs between K3 and K4') K3's rows are
  // deferred into K4' of this step (k_sim_pilot_kin<true>)
  const bool defer = allow_defer && !p.resume_nav && c->sim_re > c->sim_rb;
  MvpIn din{};
  if (mvp_device(c, p.mvp, d, (const unsigned *)c->rowoff.p, gate, sticky,
                 p.resume_nav ? nullptr : (const uint8_t *)c->inconf.p, (uint8_t *)c->s_active.p, p.reso != 0,
                 c->fuse_done, defer ? &din : nullptr))
    return -1;
  if (defer) {
    c->mvp_defer.resize(sizeof(MvpIn));
    memcpy(c->mvp_defer.data(), &din, sizeof(MvpIn));
    c->mvp_deferred = true;
  }
  // second half: resopairs rewrite, ResumeNav's asas.active, unique / cumulative counts
  return p.resume_nav ? bk_apply(c, bk) : 0;
}

// An aborted CD call (ctl = sim_ctl words [16, 48): sticky, steps done,
// resopairs demand, key-block demand): grow what overflowed on THIS rank (the
// gate is all-reduced, so every rank aborted at the same step; another rank's
// overflow re-runs the step here with unchanged buffers)
static int grow_after_abort(Ctx *c, const unsigned long long *ctl) {
  c->reuse_valid = false;  // the re-run rebuilds any reused candidate list
  c->tpr_valid = false;    // ... and any kept tile-pair list / halo plan (every rank aborted alike)
  c->zeroed_rows = -1;     // ... and zeroes every per-detect buffer (an aborted K2 wrote no inconf / tcpamax)
  {
    Counters h;
    BSA_HIP(c, hipMemcpy(&h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost));
    if (h.halo_miss)
      return fail(c, "internal error: the halo exchange and the tile-pair cull disagree (rank %d)", c->rank);
  }
  // several ranks: every rank takes part in the capacity agreement (collective)
  if (c->halo_mode == 1 && halo_grow(c)) return -1;
  if (ctl[2] > 0)  // this rank's resopairs outgrew their buffer
    c->bk_cap = std::max(2 * c->bk_cap, ctl[2] + ctl[2] / 4 + 1024);
  // pair keys outgrew their all-gather block on some rank: the block width is
  // part of the all-gather's layout, so every rank grows to the same width
  // (max-all-reduced demand; collective, every rank aborted at this step)
  // (with HK's stale flag: the device-decided stretch after a stale abort must
  // be the same on every rank -- the kept and the rebuilt plans issue
  // different collectives)
  double agree[2] = {(double)ctl[3], ctl[4] ? 1.0 : 0.0};
  if (comm_multi(c) && comm_allreduce_host(c, agree, 2, true)) return -1;
  const double kdem = agree[0];
  if (agree[1] > 0.0) {  // an HK-kept list no longer covered some rank's records: device-decided for a while
    c->hk_stale++;
    c->hk_cool = c->hk_cool_len;
    c->hk_cool_len = std::min<int64_t>(2 * c->hk_cool_len, 4096);
  }
  if (kdem > 0)
    c->bk_kw = std::max<unsigned long long>(2 * c->bk_kw, (unsigned long long)kdem + (unsigned long long)kdem / 4 + 1024);
  // candidate overflow on this rank: enough for the last detect's demand (its
  // shard counters keep counting past the capacity; every detect after the
  // abort ran on the same, unchanged state)
  Counters h;
  BSA_HIP(c, hipMemcpy(&h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost));
  static const bool trace = getenv("BSA_HK_TRACE") && atoi(getenv("BSA_HK_TRACE")) == 1;  // (diagnostics)
  if (trace)
    fprintf(stderr, "[bsa hk] rank %d abort at step %lld: stale %d k2 %llu fuse %llu halo %llu/%llu\n", c->rank,
            (long long)c->sim_steps, ctl[4] ? 1 : 0, h.k2_demand, h.fuse_ovf, h.halo_ovf, h.halo_miss);
  if (h.k2_demand) grow_k2_bucket(c, h.k2_demand);  // a K2 row bucket was full on this rank
  if (h.fuse_ovf) {  // fused K1b out of flush records: the re-run's detect unfused
    c->fuse_skip = true;
    c->fuse_retries++;
  }
  unsigned long long worst = 0;
  for (int q = 0; q < kCandShards; ++q) worst = std::max(worst, h.cshard[q][0]);
  if (worst > c->cand_cap / kCandShards)
    c->cand_cap = std::max(2 * c->cand_cap, (unsigned long long)kCandShards * (worst + worst / 4 + 1024));
  return 0;
}

static int check_params(Ctx *c, const bsa_sim_params *p) {
  if (p->cd_every < 1) return fail(c, "cd_every must be >= 1");
  if (p->resume_nav != 0 && p->resume_nav != 1) return fail(c, "resume_nav must be 0 or 1");
  if (p->winddim < 0 || p->winddim > 2) return fail(c, "winddim must be 0, 1 or 2");
  if (p->reso != 0 && p->reso != 1) return fail(c, "reso must be 0 or 1");
  return 0;
}

}  // namespace bsa

using bsa::Ctx;

extern "C" {

int bsa_sim_init(bsa_ctx *cc, int64_t n, const bsa_sim_state *s, const bsa_sim_params *p) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!s || !p) return bsa::fail(c, "NULL sim state / params");
  // every parameter is checked before anything is uploaded; a failed init
  // leaves no half-initialised sim behind (sim_ready stays false)
  c->sim_ready = false;
  if (n <= 0 || n > 0x7fffffff) return bsa::fail(c, "bad n");
  if (bsa::check_params(c, p)) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  const double *src[] = {s->lat, s->lon, s->alt, s->tas, s->hdg, s->vs, s->gs, s->trk, s->gseast,
                         s->gsnorth, s->ap_trk, s->ap_tas, s->ap_alt, s->ap_vs, s->selalt, s->bank,
                         s->eps, s->accel, s->asas_alt};
  for (auto q : src)
    if (!q) return bsa::fail(c, "bsa_sim_init: NULL array");
  // aircraft-index order first: the home order is the spatial order of this state
  if (bsa_set_state(cc, n, s->lat, s->lon, s->trk, s->gs, s->alt, s->vs)) return -1;
  if (bsa::home_order(c, p->tla, c->h2id_h)) return -1;
  bsa::set_rank_rows(c);
  if (bsa::set_home_maps(c)) return -1;
  // the all-gathered arrays hold nranks x rpr entries (in-place all-gather)
  const size_t NG = (size_t)std::max<int64_t>(n, c->sim_rpr * c->nranks) * 8;
  for (int k = 0; k < 6; ++k)
    if (!bsa::ensure_keep(c, c->own[k], NG, "gathered state")) return -1;
  std::vector<char> tmp;
  const double *st6[6] = {s->lat, s->lon, s->trk, s->gs, s->alt, s->vs};
  for (int k = 0; k < 6; ++k)
    if (bsa::put_home(c, c->own[k].p, st6[k], 8, tmp)) return -1;
  bsa::DevBuf *dst[] = {&c->s_tas, &c->s_hdg, &c->s_gse, &c->s_gsn, &c->s_aptrk, &c->s_aptas,
                        &c->s_apalt, &c->s_apvs, &c->s_selalt, &c->s_bank, &c->s_eps, &c->s_accel,
                        &c->s_aalt};
  const double *hs[] = {s->tas, s->hdg, s->gseast, s->gsnorth, s->ap_trk, s->ap_tas, s->ap_alt,
                        s->ap_vs, s->selalt, s->bank, s->eps, s->accel, s->asas_alt};
  const size_t N8 = (size_t)n * 8;
  for (int k = 0; k < 13; ++k) {
    if (!bsa::ensure(c, *dst[k], k < 4 ? NG : N8, "sim state")) return -1;
    if (bsa::put_home(c, dst[k]->p, hs[k], 8, tmp)) return -1;
  }
  // ASAS arrays: asas.trk/tas start at traf.trk/tas (asas.py:405-409), vs 0, inactive
  if (!bsa::ensure(c, c->s_atrk, N8, "asas trk") || !bsa::ensure(c, c->s_atas, N8, "asas tas") ||
      !bsa::ensure(c, c->s_avs, N8, "asas vs") || !bsa::ensure(c, c->s_ase, (size_t)n * 4, "asase") ||
      !bsa::ensure(c, c->s_asn, (size_t)n * 4, "asasn") || !bsa::ensure(c, c->s_active, n, "active") ||
      !bsa::ensure(c, c->s_altprev, N8, "pre-step altitude") || !bsa::ensure(c, c->s_ax, N8, "ax") ||
      !bsa::ensure(c, c->s_dropped, n, "ResumeNav drops"))
    return -1;
  BSA_HIP(c, hipMemsetAsync(c->s_dropped.p, 0, n, c->stream));
  c->sim_noreso = c->sim_resooff = false;  // empty NORESO / RESOOFF lists
  c->sim_atmos = false;
  BSA_HIP(c, hipMemsetAsync(c->s_ax.p, 0, N8, c->stream));   // traf.ax: 0 at create
  c->sim_limits = false;
  c->sim_perf = false;
  if (bsa::put_home(c, c->s_atrk.p, s->trk, 8, tmp) || bsa::put_home(c, c->s_atas.p, s->tas, 8, tmp)) return -1;
  BSA_HIP(c, hipMemsetAsync(c->s_avs.p, 0, N8, c->stream));
  BSA_HIP(c, hipMemsetAsync(c->s_ase.p, 0, (size_t)n * 4, c->stream));
  BSA_HIP(c, hipMemsetAsync(c->s_asn.p, 0, (size_t)n * 4, c->stream));
  BSA_HIP(c, hipMemsetAsync(c->s_active.p, 0, n, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  if (!bsa::ensure(c, c->sim_ctl, 64, "sim control words")) return -1;
  BSA_HIP(c, hipMemsetAsync(c->sim_ctl.p, 0, 64, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  c->simp = *p;
  c->bk_ready = false;  // empty resopairs / previous pair sets
  // several ranks: halo exchange instead of the full all-gather, with exact
  // initial capacities (every rank holds the whole state now)
  c->halo_mode = c->nranks > 1 ? 1 : 0;
  if (bsa::halo_init_caps(c)) return -1;
  c->sim_steps = c->sim_cd_calls = c->sim_last_conf = c->sim_last_los = 0;
  c->sim_gathered = true;
  c->sim_prepped = false;
  c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
  c->hk_ok = false;      // (HK: no build history yet)
  c->hk_cool = 0;
  c->hk_cool_len = 32;
  if (!c->hk_host) {     // HK: the pinned ring the steps' K4' publish their predictions into
    void *hp = nullptr;
    BSA_HIP(c, hipHostMalloc(&hp, (size_t)bsa::kHkRing * 8, hipHostMallocMapped | hipHostMallocCoherent));
    memset(hp, 0, (size_t)bsa::kHkRing * 8);
    c->hk_host = (unsigned long long *)hp;
    void *dp = nullptr;
    BSA_HIP(c, hipHostGetDevicePointer(&dp, hp, 0));
    c->hk_hdev = (unsigned long long *)dp;
  }
  c->sim_gs_derivable = false;  // gseast / gsnorth are the host's until K4' runs
  if (c->feed_pending) {  // a snapshot of the previous sim is dropped
    BSA_HIP(c, hipEventSynchronize(c->feed_ev));
    c->feed_pending = false;
  }
  c->home = true;
  c->sim_ready = true;
  return 0;
}

int bsa_sim_step(bsa_ctx *cc, int nsteps) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_step before bsa_sim_init");
  if (c->simp.winddim == 2 && c->wf_nvec < 1)
    return bsa::fail(c, "winddim 2 needs a wind field (bsa_set_windfield)");
  if (nsteps < 0) return bsa::fail(c, "negative step count");
  BSA_HIP(c, hipSetDevice(c->device));
  const int64_t rb = c->sim_rb, re = c->sim_re;
  const int64_t target = c->sim_steps + nsteps;
  for (int attempt = 0; c->sim_steps < target; ++attempt) {
    if (attempt > 6) return bsa::fail(c, "candidate buffer overflow in the resident step (retries exhausted)");
    const int64_t base = c->sim_steps, base_cd = c->sim_cd_calls;
    const bool derivable0 = c->sim_gs_derivable;
    BSA_HIP(c, hipMemsetAsync((char *)c->sim_ctl.p + bsa::kSimCtlSticky, 0, 40, c->stream));  // sticky, steps_done, demands, stale
    while (c->sim_steps < target) {
      bool cd_step = false;
      if (c->sim_steps % c->simp.cd_every == 0) {
        // one rank: K2 and this step's K4' as one launch (k24_launch below;
        // BSA_K24=0 off) -- K4' then starts on each workgroup's rows as soon as
        // their fold is done, instead of behind the whole of K2
        static const bool k24_env = !(getenv("BSA_K24") && atoi(getenv("BSA_K24")) == 0);
        c->k24_want = k24_env && c->nranks == 1 && c->halo_mode == 0 && !c->simp.resume_nav && re > rb &&
                      c->k2_bucket > 0;
        c->hk_req = true;  // (HK: this detect's list decision may be the host's)
        const int r = bsa::sim_cd(c, true);
        c->hk_req = false;
        c->k24_want = false;
        if (r) {
          c->k24_pending = false;
          c->hk_ok = false;  // (a detect may have been enqueued without its step's publication)
          return -1;
        }
        cd_step = true;
      }
      // K4' workgroup size: one wave (at 100k rows 256-lane groups left half the
      // CUs one group short, 391 groups on 256 CUs: 0.1753 -> 0.1718 ms per
      // step with 64; BSA_K4_BLOCK=128/256 for A/B)
      static const int k4b = [] {
        const int v = getenv("BSA_K4_BLOCK") ? atoi(getenv("BSA_K4_BLOCK")) : 64;
        return (v == 64 || v == 128 || v == 256) ? v : 64;
      }();
      // one rank, the next step a CD step: K4' also prepares that detect's
      // column records and boxes (its K0b launch is skipped; BSA_SIM_PREP=0 off)
      static const bool prep_env = !(getenv("BSA_SIM_PREP") && atoi(getenv("BSA_SIM_PREP")) == 0);
      const bool prep = prep_env && c->nranks == 1 && c->home && !c->reuse_on && c->halo_mode == 0 && rb == 0 &&
                        re == c->n && (c->sim_steps + 1) % c->simp.cd_every == 0;
      bsa::PrepArgs pa{};
      if (prep) {
        const int64_t n = c->n;
        pa.rec = bsa::home_records(c, n) ? 1 : 0;
        if ((pa.rec && !bsa::ensure(c, c->colrec, n * sizeof(bsa::ColRec), "column records")) ||
            !bsa::ensure(c, c->pfcol, n * sizeof(bsa::PFRec), "prefilter columns") ||
            !bsa::ensure(c, c->pfvcol, n * sizeof(bsa::PFVel), "prefilter column velocities") ||
            !bsa::ensure(c, c->pfpcol, n * sizeof(float4), "prefilter column positions") ||
            !bsa::ensure(c, c->tbox_c, ((n + bsa::kTile - 1) / bsa::kTile) * sizeof(bsa::TileBox), "column tile boxes") ||
            !bsa::ensure(c, c->gbox_c, ((n + bsa::kGroup - 1) / bsa::kGroup) * sizeof(bsa::TileBox), "column group boxes") ||
            !bsa::ensure(c, c->sbox_c, ((n + bsa::kSub - 1) / bsa::kSub) * sizeof(bsa::TileBox), "column sub-group boxes"))
          return -1;
        pa.out = bsa::PrepOut{(bsa::ColRec *)c->colrec.p, (bsa::PFRec *)c->pfcol.p, (bsa::PFVel *)c->pfvcol.p,
                              (float4 *)c->pfpcol.p};
        pa.sbox = (bsa::TileBox *)c->sbox_c.p;
        pa.gbox = (bsa::TileBox *)c->gbox_c.p;
        pa.rpz = c->simp.rpz;
        pa.hpz = c->simp.hpz;
        pa.tla = c->simp.tla;
        pa.mid = bsa::stage1_mid(0, false, 0);
        pa.n = (int)n;
        if (!bsa::nonfin_word(c)) return -1;
        pa.nf = (unsigned long long *)c->nonfin.p;  // the next detect's records: a fresh epoch
        pa.nfe = c->nf_prep_epoch = ++c->nf_counter;
        if (c->tpr_valid && c->tpr_snap.p && c->tpr_ctl.p && c->tpr_n == n) {  // the kept list's budgets
          pa.snap = (const bsa::PFRec *)c->tpr_snap.p;
          pa.tpr_ctl = (unsigned long long *)c->tpr_ctl.p;
          pa.dx = c->tpr_dx;
          pa.ds = c->tpr_ds;
          pa.dv = c->tpr_dv;
          // HK: the prediction word of the next detect (index hk_m, if it is host-decided)
          pa.pred = (unsigned long long *)c->tpr_ctl.p + 6 + (c->hk_m & 1);
          pa.pf = c->hk_f;
        }
      }
      const int blk = k4b;  // (PREP: whole waves = whole groups, rb = 0)
      const int64_t nb = std::max<int64_t>(1, (re - rb + blk - 1) / blk);
      bsa::MvpIn mv{};
      if (c->mvp_deferred) memcpy(&mv, c->mvp_defer.data(), sizeof(mv));
      // HK: the CD step's K4' (or K2 + K4') publishes the detect's prediction --
      // the rank's own word with K2 fused, else gate[2] after K2 and the all-reduce
      bsa::HkPub pub{};
      if (cd_step && c->hk_cur) {
        pub.slot = c->hk_hdev + (c->hk_last % bsa::kHkRing);
        pub.base = (unsigned long long)(c->hk_last + 1) << 2;
        if (c->k24_pending) {
          pub.src = (unsigned long long *)c->tpr_ctl.p + 6 + (c->hk_last & 1);
          pub.zero = 1;
        } else {
          pub.src = (unsigned long long *)c->sim_ctl.p + 2;
        }
      }
      if (c->k24_pending) {  // K2 of this step's detect, fused with K4' (double-buffered alt / vs / gse / gsn)
        const int64_t n = c->n;
        if (!c->mvp_deferred) return bsa::fail(c, "internal: fused K2 + K4' without the deferred MVP rows");
        if (!bsa::ensure(c, c->nx_alt, n * 8, "next altitudes") || !bsa::ensure(c, c->nx_vs, n * 8, "next vs") ||
            !bsa::ensure(c, c->nx_gse, n * 8, "next gseast") || !bsa::ensure(c, c->nx_gsn, n * 8, "next gsnorth"))
          return -1;
        bsa::SimDev d = bsa::sim_dev(c);
        d.alt_w = (double *)c->nx_alt.p;
        d.vs_w = (double *)c->nx_vs.p;
        d.gse_w = (double *)c->nx_gse.p;
        d.gsn_w = (double *)c->nx_gsn.p;
        const bsa::K24Args ka{d, mv, c->simp.mvp, pa, bsa::wind_field(c), c->simp.simdt, c->simp.windnorth,
                              c->simp.windeast, c->simp.winddim, prep ? 1 : 0, pub};
        if (bsa::k24_launch(c, ka)) return -1;
        std::swap(c->own[4], c->nx_alt);
        std::swap(c->own[5], c->nx_vs);
        std::swap(c->s_gse, c->nx_gse);
        std::swap(c->s_gsn, c->nx_gsn);
      } else {
        const auto K4 = c->mvp_deferred ? (prep ? bsa::k_sim_pilot_kin<true, true> : bsa::k_sim_pilot_kin<true, false>)
                                        : (prep ? bsa::k_sim_pilot_kin<false, true> : bsa::k_sim_pilot_kin<false, false>);
        hipLaunchKernelGGL(K4, dim3((unsigned)nb), dim3(blk), 0, c->stream, (int)rb, (int)re, c->simp.simdt,
                           c->simp.winddim, c->simp.windnorth, c->simp.windeast, bsa::wind_field(c), bsa::sim_dev(c),
                           mv, c->simp.mvp, pa, pub);
      }
      c->mvp_deferred = false;
      c->sim_prepped = prep;
      if (prep) {
        c->sim_prep_key[0] = pa.rpz;
        c->sim_prep_key[1] = pa.hpz;
        c->sim_prep_key[2] = pa.tla;
        c->sim_prep_key[3] = (double)pa.mid;
        c->sim_prep_n = c->n;
      }
      BSA_HIP(c, hipGetLastError());
      // every rank's rows now hold K4's gs / trk / gse / gsn: gse / gsn follow
      // from gs / trk bitwise only without wind (with wind gs / trk derive from
      // them, traffic.py:463-466, not the other way round)
      c->sim_gs_derivable = c->simp.winddim == 0;
      c->sim_gathered = c->nranks == 1;
      c->sim_steps++;
    }
    // the batch's only host synchronisation: did every step complete?
    unsigned long long ctl[5] = {0, 0, 0, 0, 0};
    BSA_HIP(c, hipMemcpyAsync(ctl, (char *)c->sim_ctl.p + bsa::kSimCtlSticky, 40, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
#ifdef BSA_PF_TRACE
    if (bsa::pf_trace_dump(c, 0, 0)) return -1;  // (diagnostic builds: the batch's last prefilter)
#endif
    if ((unsigned)ctl[0] == 0) break;
    // aborted at step base + done: the state is that of the step's start.  The
    // gate is all-reduced, so every rank aborted at the same step; each rank
    // grows only the buffers that overflowed on IT (another rank's overflow
    // re-runs the step with unchanged buffers here) and all ranks re-run it
    c->reuse_valid = false;  // the re-run rebuilds any reused candidate list
    c->sim_prepped = false;  // (an aborted K4' prepared nothing)
    c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
    c->hk_ok = false;      // (HK: the decisions of the aborted steps never took effect)
    const int64_t done = (int64_t)ctl[1];
    c->sim_steps = base + done;
    c->sim_gs_derivable = done > 0 ? c->simp.winddim == 0 : derivable0;  // K4' ran for the completed steps only
    int64_t cds = 0;
    for (int64_t k = base; k < base + done; ++k) cds += (k % c->simp.cd_every == 0) ? 1 : 0;
    c->sim_cd_calls = base_cd + cds;
    c->sim_gathered = c->nranks == 1;
    if (bsa::grow_after_abort(c, ctl)) return -1;
  }
  return 0;
}

int bsa_sim_set_limits(bsa_ctx *cc, const double *hmax, const double *vmin, const double *vmax,
                       const double *vsmin, const double *vsmax, const double *axmax) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_set_limits before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  if (!hmax) {
    c->sim_limits = false;
    return 0;
  }
  const double *src[6] = {hmax, vmin, vmax, vsmin, vsmax, axmax};
  for (auto q : src)
    if (!q) return bsa::fail(c, "bsa_sim_set_limits: NULL envelope array");
  const size_t N8 = (size_t)c->n * 8;
  if (!bsa::ensure(c, c->s_env, 6 * N8, "OpenAP envelope")) return -1;
  std::vector<char> tmp;
  for (int k = 0; k < 6; ++k)
    if (bsa::put_home(c, (char *)c->s_env.p + k * N8, src[k], 8, tmp)) return -1;
  c->sim_limits = true;
  return 0;
}

int bsa_sim_set_perf(bsa_ctx *cc, int64_t ntypes, const double *table, const int32_t *type_idx) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_set_perf before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  if (!table) {
    c->sim_perf = false;
    return 0;
  }
  if (ntypes < 1 || !type_idx) return bsa::fail(c, "bsa_sim_set_perf: bad type table");
  // every index and lift type is checked here: the kernel reads the table unguarded
  for (int64_t t = 0; t < ntypes; ++t) {
    const double lt = table[t * bsa::kin::kPerfCols + 22];
    if (lt != 0.0 && lt != 1.0 && lt != 2.0) return bsa::fail(c, "type %lld: lifttype must be 0, 1 or 2", (long long)t);
  }
  const int64_t n = c->n;
  for (int64_t k = 0; k < n; ++k)
    if (type_idx[k] < 0 || type_idx[k] >= ntypes)
      return bsa::fail(c, "aircraft %lld: type index %d outside [0, %lld)", (long long)k, type_idx[k], (long long)ntypes);
  const size_t tb = (size_t)ntypes * bsa::kin::kPerfCols * 8;
  if (!bsa::ensure(c, c->s_ptab, tb, "OpenAP type table") || !bsa::ensure(c, c->s_ptype, (size_t)n * 4, "type index") ||
      !bsa::ensure(c, c->s_phase, (size_t)n, "flight phase"))
    return -1;
  BSA_HIP(c, hipMemcpyAsync(c->s_ptab.p, table, tb, hipMemcpyHostToDevice, c->stream));
  std::vector<char> tmp;
  if (bsa::put_home(c, c->s_ptype.p, type_idx, 4, tmp)) return -1;
  BSA_HIP(c, hipMemsetAsync(c->s_phase.p, 0, (size_t)n, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  c->sim_perf = true;
  c->sim_ntypes = ntypes;
  return 0;
}

int bsa_sim_read_perf(bsa_ctx *cc, uint8_t *phase, double *ax) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_read_perf before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<char> tmp;
  if (phase) {
    if (!c->sim_perf) return bsa::fail(c, "no flight phase: bsa_sim_set_perf is off");
    if (bsa::get_home(c, phase, c->s_phase.p, 1, c->sim_rb, c->sim_re, tmp)) return -1;
  }
  if (ax && bsa::get_home(c, ax, c->s_ax.p, 8, c->sim_rb, c->sim_re, tmp)) return -1;
  return 0;
}

int bsa_sim_update(bsa_ctx *cc, const bsa_sim_state *s) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!s) return bsa::fail(c, "NULL sim state");
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_update before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  struct {
    const double *src;
    void *dst;
  } cp[] = {{s->lat, c->own[0].p},     {s->lon, c->own[1].p},     {s->trk, c->own[2].p},
            {s->gs, c->own[3].p},      {s->alt, c->own[4].p},     {s->vs, c->own[5].p},
            {s->tas, c->s_tas.p},      {s->hdg, c->s_hdg.p},      {s->gseast, c->s_gse.p},
            {s->gsnorth, c->s_gsn.p},  {s->ap_trk, c->s_aptrk.p}, {s->ap_tas, c->s_aptas.p},
            {s->ap_alt, c->s_apalt.p}, {s->ap_vs, c->s_apvs.p},   {s->selalt, c->s_selalt.p},
            {s->bank, c->s_bank.p},    {s->eps, c->s_eps.p},      {s->accel, c->s_accel.p},
            {s->asas_alt, c->s_aalt.p}};
  // the replicated CD inputs are rewritten on every rank (in the sim's home order)
  bool any_cd = false, all_rep = true;
  bsa::HomeBatch hb(c, true);
  for (int k = 0; k < 19; ++k) {
    const bool rep = k < 6 || k == 8 || k == 9;  // the arrays the all-gather replicates
    if (!cp[k].src) {
      all_rep = all_rep && !rep;
      continue;
    }
    if (k < 10) any_cd = true;
    if (hb.add(cp[k].dst, cp[k].src, nullptr, 8)) return -1;
  }
  if (hb.run()) return -1;
  c->sim_prepped = false;  // prepared records are of the old state
  c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
  if (any_cd) {
    // every rank passed the same full arrays: the replicas are consistent only
    // if ALL replicated arrays were passed; otherwise the next all-gather
    // repairs the other ranks' rows of the arrays not passed (each rank's
    // own rows are right either way)
    if (all_rep) c->sim_gathered = true;
    c->sim_gs_derivable = false;  // (gseast / gsnorth may be the host's)
    c->reuse_valid = false;       // a state jump rebuilds any reused candidate list
  }
  return 0;
}

int bsa_sim_read(bsa_ctx *cc, bsa_sim_out *o) {
  Ctx *c = (Ctx *)cc;
  if (!c || !o) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_read before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  if (bsa::sim_gather(c) || bsa::sim_gather_asas(c)) return -1;
  struct {
    void *dst;
    const void *src;
    size_t esz;
  } cp[] = {{o->lat, c->own[0].p, 8},      {o->lon, c->own[1].p, 8},      {o->alt, c->own[4].p, 8},
            {o->tas, c->s_tas.p, 8},       {o->hdg, c->s_hdg.p, 8},       {o->vs, c->own[5].p, 8},
            {o->gs, c->own[3].p, 8},       {o->trk, c->own[2].p, 8},      {o->gseast, c->s_gse.p, 8},
            {o->gsnorth, c->s_gsn.p, 8},   {o->asas_trk, c->s_atrk.p, 8}, {o->asas_tas, c->s_atas.p, 8},
            {o->asas_vs, c->s_avs.p, 8},   {o->asas_alt, c->s_aalt.p, 8},
            {o->active, c->s_active.p, 1}};
  bsa::HomeBatch hb(c, false);
  for (auto &e : cp)
    if (e.dst && hb.add(const_cast<void *>(e.src), nullptr, e.dst, (int)e.esz)) return -1;
  return hb.run();
}

int bsa_sim_stats(bsa_ctx *cc, int64_t *out6) {
  Ctx *c = (Ctx *)cc;
  if (!c || !out6) return -1;
  if (c->sim_cd_calls > 0 && c->counters.p) {  // counts of the last CD step
    BSA_HIP(c, hipSetDevice(c->device));
    bsa::Counters h;
    BSA_HIP(c, hipMemcpyAsync(&h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    c->sim_last_conf = (int64_t)h.conf;
    c->sim_last_los = (int64_t)h.los;
  }
  out6[0] = c->sim_steps;
  out6[1] = c->sim_cd_calls;
  out6[2] = c->sim_last_conf;
  out6[3] = c->sim_last_los;
  out6[4] = c->sim_rb;
  out6[5] = c->sim_re;
  return 0;
}

int bsa_sim_detect_rows(bsa_ctx *cc, int64_t row_begin, int64_t row_end, int64_t *n_conf, int64_t *n_los) {
  Ctx *c = (Ctx *)cc;
  if (!c || !n_conf || !n_los) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_detect_rows before bsa_sim_init");
  if (row_begin % bsa::kTile != 0) return bsa::fail(c, "row_begin must be a multiple of %d", bsa::kTile);
  BSA_HIP(c, hipSetDevice(c->device));
  if (bsa::sim_gather(c)) return -1;
  // as one rank of a sharded step: own tiles, halo plan, halo tiles (the
  // boxes of every tile, which the other ranks would send, are prepared
  // first, outside the detect's timed stages).  Those records carry the
  // detect's non-finite epoch: a NaN column outside this share's halo makes
  // every row's tcpamax NaN, as in the whole detect (StateBasedCD.py:90; the
  // sharded step carries it through the gate all-reduce instead)
  if (!bsa::nonfin_word(c)) return -1;
  const unsigned long long e = ++c->nf_counter;
  if (bsa::prep_all_tiles(c, c->simp.rpz, c->simp.hpz, c->simp.tla, e)) return -1;
  const int hm = c->halo_mode;
  c->halo_mode = 2;
  c->det_home = true;
  c->nf_force_epoch = e;  // (retries of the detect too)
  const int r = bsa::detect(c, c->simp.rpz, c->simp.hpz, c->simp.tla, 0, row_begin, row_end, n_conf, n_los);
  c->nf_force_epoch = 0;
  c->det_home = false;
  c->halo_mode = hm;
  return r;
}

int bsa_sim_probe_rank(bsa_ctx *cc, int rank, int nranks) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_probe_rank before bsa_sim_init");
  if (c->nranks != 1) return bsa::fail(c, "bsa_sim_probe_rank: a one-rank sim only (it plays one rank of several)");
  if (nranks < 1 || rank < 0 || rank >= nranks) return bsa::fail(c, "bad probe rank %d of %d", rank, nranks);
  BSA_HIP(c, hipSetDevice(c->device));
  const int64_t n = c->n;
  c->tpr_valid = false;  // (its tile-pair list / plan are rebuilt for the new rows)
  c->sim_prepped = false;
  if (nranks == 1) {  // back to the whole sim
    c->sim_rb = 0;
    c->sim_re = n;
    c->halo_mode = 0;
    return bsa::set_home_maps(c);  // (the rows' index order: row ids, fetched pairs)
  }
  // the rank's home range (bsa_sim_init's partition) and the one-GPU halo
  // mode of bsa_sim_detect_rows: the other ranks' tiles are prepared once here
  // (their rows do not move: only this rank's K4' runs), the rank's own tiles
  // and its halo by every detect
  const int64_t rpr = ((n + nranks - 1) / nranks + bsa::kTile - 1) / bsa::kTile * bsa::kTile;
  c->sim_rb = std::min<int64_t>(n, (int64_t)rank * rpr);
  c->sim_re = std::min<int64_t>(n, c->sim_rb + rpr);
  if (c->sim_rb % bsa::kTile != 0) return bsa::fail(c, "probe rank %d of %d holds no rows", rank, nranks);
  if (bsa::set_home_maps(c) || bsa::sim_gather(c) || bsa::prep_all_tiles(c, c->simp.rpz, c->simp.hpz, c->simp.tla))
    return -1;
  c->halo_mode = 2;
  return 0;
}

int bsa_sim_halo_stats(bsa_ctx *cc, int64_t *out4) {
  Ctx *c = (Ctx *)cc;
  if (!c || !out4) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  unsigned tiles = 0;
  if (c->h_dem.p) {  // the received-tile total of the last plan (after its demand words)
    BSA_HIP(c, hipMemcpyAsync(&tiles, (const unsigned *)c->h_dem.p + c->halo_tot_word, 4, hipMemcpyDeviceToHost,
                              c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
  }
  out4[0] = c->halo_rx;
  out4[1] = c->halo_tx;
  out4[2] = tiles;
  out4[3] = c->halo_grows;
  return 0;
}

int bsa_sim_set_halo_cap(bsa_ctx *cc, int sender, int receiver, int64_t tiles) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  const int R = c->nranks;
  if ((int64_t)c->halo_cap.size() != (int64_t)R * R) return bsa::fail(c, "no halo capacities (one rank, or no sim)");
  if (sender < 0 || sender >= R || receiver < 0 || receiver >= R || sender == receiver || tiles < 0)
    return bsa::fail(c, "bad halo capacity %d -> %d = %lld", sender, receiver, (long long)tiles);
  c->halo_cap[(size_t)sender * R + receiver] = tiles;
  return 0;
}

int bsa_sim_halo_recheck(bsa_ctx *cc) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  c->halo_chk_gen = -1;  // (collective by contract: every rank calls it before the same step)
  return 0;
}

int bsa_sim_row_ids(bsa_ctx *cc, int32_t *ids) {
  Ctx *c = (Ctx *)cc;
  if (!c || !ids) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_row_ids before bsa_sim_init");
  const int64_t rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  for (int64_t r = 0; r < nr; ++r) ids[c->lpos_h[(size_t)r]] = (int32_t)c->h2id_h[(size_t)(rb + r)];
  return 0;
}

int bsa_sim_asas_stats(bsa_ctx *cc, int64_t *out6) {
  Ctx *c = (Ctx *)cc;
  if (!c || !out6) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_asas_stats before bsa_sim_init");
  if (!c->simp.resume_nav) return bsa::fail(c, "ASAS bookkeeping is off (resume_nav = 0)");
  BSA_HIP(c, hipSetDevice(c->device));
  unsigned long long st[8] = {0};
  if (c->bk_ready) BSA_HIP(c, hipMemcpyAsync(st, c->bk_stats.p, 64, hipMemcpyDeviceToHost, c->stream));
  const int64_t rb = c->sim_rb, nr = c->sim_re - c->sim_rb;
  std::vector<uint8_t> act((size_t)std::max<int64_t>(nr, 1));
  if (nr > 0) BSA_HIP(c, hipMemcpyAsync(act.data(), (uint8_t *)c->s_active.p + rb, nr, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  int64_t na = 0;
  for (int64_t k = 0; k < nr; ++k) na += act[k] ? 1 : 0;
  out6[0] = (int64_t)st[0];
  for (int k = 1; k < 5; ++k) out6[k] = (int64_t)st[k];  // global sets (identical on every rank)
  out6[5] = na;
  return 0;
}

int bsa_sim_resopairs(bsa_ctx *cc, int32_t *idx1, int32_t *idx2, int64_t cap, int64_t *count) {
  Ctx *c = (Ctx *)cc;
  if (!c || !count) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_resopairs before bsa_sim_init");
  if (!c->simp.resume_nav) return bsa::fail(c, "ASAS bookkeeping is off (resume_nav = 0)");
  if (cap > 0 && (!idx1 || !idx2)) return bsa::fail(c, "NULL resopairs buffer");
  BSA_HIP(c, hipSetDevice(c->device));
  *count = 0;
  if (!c->bk_ready) return 0;
  const int64_t nr = c->last_re - c->last_rb;
  std::vector<unsigned> ptr((size_t)nr + 1);
  BSA_HIP(c, hipMemcpyAsync(ptr.data(), c->bk_rptr.p, (size_t)(nr + 1) * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  const int64_t total = ptr[(size_t)nr];
  *count = total;
  if (total > cap || total == 0) return 0;
  std::vector<unsigned> col((size_t)total);
  BSA_HIP(c, hipMemcpyAsync(col.data(), c->bk_rcol.p, (size_t)total * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  // rows in ascending aircraft index (each row's columns are ascending, a
  // deleted intruder's marker last)
  std::vector<unsigned> ord((size_t)nr);
  for (int64_t r = 0; r < nr; ++r) ord[(size_t)r] = (unsigned)r;
  const unsigned *H = c->h2id_h.data() + c->last_rb;
  std::sort(ord.begin(), ord.end(), [&](unsigned a, unsigned b) { return H[a] < H[b]; });
  int64_t at = 0;
  for (unsigned r : ord)
    for (unsigned k = ptr[r]; k < ptr[r + 1]; ++k, ++at) {
      idx1[at] = (int32_t)H[r];
      idx2[at] = (int32_t)col[k];
    }
  return 0;
}

int bsa_sim_cd(bsa_ctx *cc) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_cd before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  for (int attempt = 0;; ++attempt) {
    if (attempt > 6) return bsa::fail(c, "candidate buffer overflow in the CD call (retries exhausted)");
    const int64_t base_cd = c->sim_cd_calls;
    BSA_HIP(c, hipMemsetAsync((char *)c->sim_ctl.p + bsa::kSimCtlSticky, 0, 40, c->stream));  // sticky, steps_done, demands, stale
    if (bsa::sim_cd(c, false)) return -1;
    unsigned long long ctl[5] = {0, 0, 0, 0, 0};
    BSA_HIP(c, hipMemcpyAsync(ctl, (char *)c->sim_ctl.p + bsa::kSimCtlSticky, 40, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    if ((unsigned)ctl[0] == 0) break;
    // aborted: nothing persistent was written (the state did not move, so
    // the replicas stay consistent); grow and re-run
    c->sim_cd_calls = base_cd;
    if (bsa::grow_after_abort(c, ctl)) return -1;
  }
  return 0;
}

int bsa_sim_set_params(bsa_ctx *cc, const bsa_sim_params *p) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!p) return bsa::fail(c, "NULL sim params");
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_set_params before bsa_sim_init");
  if (bsa::check_params(c, p)) return -1;
  if (p->resume_nav && !c->simp.resume_nav) c->bk_ready = false;  // the bookkeeping starts empty
  c->simp = *p;
  c->sim_prepped = false;
  c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
  return 0;
}

int bsa_sim_set_reso_lists(bsa_ctx *cc, const uint8_t *noreso, const uint8_t *resooff) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_set_reso_lists before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<char> tmp;
  struct {
    const uint8_t *h;
    bsa::DevBuf *b;
    bool *on;
  } ls[2] = {{noreso, &c->s_noreso, &c->sim_noreso}, {resooff, &c->s_resooff, &c->sim_resooff}};
  for (auto &l : ls) {
    *l.on = false;
    if (!l.h) continue;
    std::vector<uint8_t> v(l.h, l.h + c->n);
    for (auto &x : v) x = x ? 1 : 0;
    if (!bsa::ensure(c, *l.b, (size_t)c->n, "NORESO / RESOOFF list") || bsa::put_home(c, l.b->p, v.data(), 1, tmp))
      return -1;
    *l.on = true;
  }
  return 0;
}

int bsa_sim_read_asas(bsa_ctx *cc, bsa_asas_out *o) {
  Ctx *c = (Ctx *)cc;
  if (!c || !o) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_read_asas before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  struct {
    void *dst;
    const void *src;
    size_t esz;
  } cp[] = {{o->trk, c->s_atrk.p, 8},   {o->tas, c->s_atas.p, 8},     {o->vs, c->s_avs.p, 8},
            {o->alt, c->s_aalt.p, 8},   {o->asase, c->s_ase.p, 4},    {o->asasn, c->s_asn.p, 4},
            {o->active, c->s_active.p, 1}, {o->dropped, c->s_dropped.p, 1}};
  if (c->sim_rb == 0 && c->sim_re == c->n) {  // one rank: every row, one batch
    bsa::HomeBatch hb(c, false);
    for (auto &e : cp)
      if (e.dst && hb.add(const_cast<void *>(e.src), nullptr, e.dst, (int)e.esz)) return -1;
    return hb.run();
  }
  std::vector<char> tmp;
  for (auto &e : cp)
    if (e.dst && bsa::get_home(c, e.dst, e.src, e.esz, c->sim_rb, c->sim_re, tmp)) return -1;
  return 0;
}

int bsa_sim_set_atmos(bsa_ctx *cc, int on) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready) return bsa::fail(c, "bsa_sim_set_atmos before bsa_sim_init");
  BSA_HIP(c, hipSetDevice(c->device));
  if (on && !c->sim_atmos) {
    if (!bsa::ensure(c, c->s_atm, (size_t)c->n * 24, "atmosphere")) return -1;
    BSA_HIP(c, hipMemsetAsync(c->s_atm.p, 0, (size_t)c->n * 24, c->stream));
  }
  c->sim_atmos = on != 0;
  return 0;
}

int bsa_sim_read_atmos(bsa_ctx *cc, double *p, double *rho, double *temp) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!c->sim_ready || !c->sim_atmos) return bsa::fail(c, "bsa_sim_read_atmos: atmosphere outputs are off");
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<char> tmp;
  double *dst[3] = {p, rho, temp};
  for (int k = 0; k < 3; ++k)
    if (dst[k] && bsa::get_home(c, dst[k], (const char *)c->s_atm.p + (size_t)k * c->n * 8, 8, c->sim_rb, c->sim_re, tmp))
      return -1;
  return 0;
}

}  // extern "C"
