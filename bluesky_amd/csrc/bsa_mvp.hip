// K3: MVP conflict resolution on the device-resident, canonically sorted
// conflict pairs of the last detect.
//
// bluesky/traffic/asas/MVP.py:14-143 loops over confpairs and only ever
// writes dv[id1] (MVP.py:46-61; prioRules' dv2 is discarded), and confpairs
// are in row-major order, so each ownship's dv is a sequential fold over its
// own contiguous segment of pairs in j order.  Each pair's MVP vector does
// not depend on the fold, so k_mvp_pair computes them all in parallel (one
// lane per pair); k_mvp_row then folds each ownship's segment in order, which
// reproduces the reference's summation order exactly (no tree reduction),
// and runs the per-aircraft finalize (MVP.py:67-143).
#include "bsa_geo_math.h"  // np_max / np_min / np_rem
#include "bsa_internal.h"
#include "bsa_mvp_math.h"
#include "bsa_mvp_row.h"

#pragma clang fp contract(off)

namespace bsa {

// segment start of each row: first k with ci[k] >= rb + r  (ci sorted);
// seg[nrows] = P.  Used when the pairs came from the host (bsa_set_pairs);
// a device detect hands its K2 row offsets over directly.
__global__ __launch_bounds__(256) void k_segments(int nrows, int rb, int64_t P,
                                                  const int *__restrict__ ci,
                                                  unsigned *__restrict__ seg) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  const int key = rb + r;
  int64_t lo = 0, hi = P;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ci[mid] < key) lo = mid + 1; else hi = mid;
  }
  seg[r] = (unsigned)lo;
}

// Per pair (MVP.py:33-56): MVP.MVP (MVP.py:149-231) and the priority rules
// (MVP.py:235-300; only the first return value is kept, MVP.py:46) for one
// confpair.  Nothing here depends on the running dv sum, so the pairs are
// independent; k_mvp_row applies the results in the reference's order.
__global__ __launch_bounds__(256) void k_mvp_pair(int rb, bsa_mvp_params p, MvpIn in) {
  if (mvp_aborted(in) || !in.resolve) return;
  const unsigned P = in.seg[in.nrows];
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned k = blockIdx.x * blockDim.x + threadIdx.x; k < P; k += stride) {
    double4 dv;
    uint8_t fl;
    mvp_pair(p, MvpPairIn{in.gseast, in.gsnorth, in.vs, in.alt, p.swnoreso ? in.noreso : nullptr, nullptr}, in.ci[k],
             in.cj[k], in.pay[k], in.pay[(size_t)1 * P + k], in.pay[(size_t)2 * P + k],
             in.pay[(size_t)3 * P + k], dv, fl);
    in.pdv[k] = dv;
    in.pfl[k] = fl;
  }
}

// K3 per row (bsa_mvp_row.h); in the resident step it also gates the step
// (overflow -> sticky abort)
__global__ __launch_bounds__(256) void k_mvp_row(int rb, bsa_mvp_params p, MvpIn in) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (in.gate) {
    const bool abort = in.sticky[0] != 0 || in.gate[0] >= kGateOverflow;
    if (r == 0 && in.gate[0] >= kGateOverflow) in.sticky[0] = 1u;
    if (abort) return;
  }
  if (r >= in.nrows) return;
  mvp_row(rb, r, p, in);
}

// Device-side MVP over the last detect's pairs; all pointers are device
// pointers (full-N traffic arrays, per-row outputs).  seg: the detect's K2
// row offsets (device path) or NULL (pairs from the host: binary search).
// gate / sticky / inconf / active: resident sim step only.
int mvp_device(Ctx *c, const bsa_mvp_params &p, const MvpDev &d, const unsigned *seg,
               const unsigned long long *gate, unsigned *sticky, const uint8_t *inconf, uint8_t *active,
               bool resolve, bool pairs_done, MvpIn *defer) {
  const int64_t rb = c->last_rb, re = c->last_re, nrows = std::max<int64_t>(re - rb, 0);
  if (nrows == 0 && !gate) return 0;  // (a resident rank without rows still applies the gate)
  const unsigned long long pcap = std::max<unsigned long long>(c->cand_cap, (unsigned long long)c->last_conf);
  if (!ensure(c, c->mvp_pdv, std::max<unsigned long long>(pcap, 1) * sizeof(double4), "mvp pair dv") ||
      !ensure(c, c->mvp_pfl, std::max<unsigned long long>(pcap, 1), "mvp pair flags"))
    return -1;
  if (nrows == 0) {
    MvpIn in{};
    in.gate = gate;
    in.sticky = sticky;
    hipLaunchKernelGGL(k_mvp_row, dim3(1), dim3(64), 0, c->stream, (int)rb, p, in);
    BSA_HIP(c, hipGetLastError());
    return 0;
  }
  if (!seg) {
    if (!ensure(c, c->seg, (size_t)(nrows + 1) * 4, "mvp segments")) return -1;
    hipLaunchKernelGGL(k_segments, dim3((unsigned)((nrows + 1 + 255) / 256)), dim3(256), 0, c->stream,
                       (int)nrows, (int)rb, c->last_conf, (const int *)c->out_ci.p, (unsigned *)c->seg.p);
    BSA_HIP(c, hipGetLastError());
    seg = (const unsigned *)c->seg.p;
  }
  MvpIn in{};
  in.ci = (const int *)c->out_ci.p;
  in.cj = (const int *)c->out_cj.p;
  in.pay = (const double *)c->out_pay.p;
  in.seg = seg;
  in.gseast = d.gseast;
  in.gsnorth = d.gsnorth;
  in.vs = d.vs;
  in.alt = d.alt;
  in.trk = d.trk;
  in.gs = d.gs;
  in.selalt = d.selalt;
  in.apvs = d.apvs;
  in.aptrk = d.aptrk;
  in.aptas = d.aptas;
  in.apalt = d.apalt;
  in.noreso = d.noreso;
  in.resooff = d.resooff;
  in.asas_alt = d.asas_alt;
  in.o_trk = d.o_trk;
  in.o_tas = d.o_tas;
  in.o_vs = d.o_vs;
  in.o_asase = d.o_asase;
  in.o_asasn = d.o_asasn;
  in.o_tsolv = d.o_tsolv;
  in.pdv = (double4 *)c->mvp_pdv.p;
  in.pfl = (uint8_t *)c->mvp_pfl.p;
  // K2 of the same detect folded each row's vectors (k_rank_rows)
  in.rowdv = pairs_done && c->fuse_rowdv && resolve ? (const double4 *)c->mvp_rowdv.p : nullptr;
  in.gate = gate;
  in.sticky = sticky;
  in.inconf = inconf;
  in.active = active;
  in.nrows = (int)nrows;
  in.resolve = resolve ? 1 : 0;
  // several ranks: the gate's non-finite word reaches every rank's tcpamax here
  in.tcpamax = gate && comm_multi(c) ? (unsigned long long *)c->tcpamax.p : nullptr;
  if (!resolve && (!gate || !d.aptrk || !d.aptas || !d.apalt))
    return fail(c, "CR OFF (DoNothing) needs the resident step's autopilot targets");
  if (!pairs_done && resolve) {  // else K2 of the same step already wrote pdv / pfl (k_rank)
    hipLaunchKernelGGL(k_mvp_pair, dim3(256 * 4), dim3(256), 0, c->stream, (int)rb, p, in);
    BSA_HIP(c, hipGetLastError());
  }
  if (defer) {
    *defer = in;
    return 0;
  }
  hipLaunchKernelGGL(k_mvp_row, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, c->stream, (int)rb, p,
                     in);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

}  // namespace bsa

// ---------------------------------------------------------------- C ABI (host buffers)
extern "C" int bsa_mvp(bsa_ctx *cc, const bsa_mvp_params *p, const double *gseast,
                       const double *gsnorth, const double *selalt, const double *apvs,
                       const uint8_t *noreso, const uint8_t *resooff, double *asas_alt,
                       double *trk, double *tas, double *vs, float *asase, float *asasn) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  if (!p) return bsa::fail(c, "NULL params");
  if (!gseast || !gsnorth || !selalt || !apvs || !asas_alt || !trk || !tas || !vs || !asase || !asasn)
    return bsa::fail(c, "bsa_mvp: NULL array argument");
  BSA_HIP(c, hipSetDevice(c->device));
  if (!c->have_pairs) return bsa::fail(c, "bsa_mvp: no detect results (call bsa_detect first)");
  if (c->home) return bsa::fail(c, "bsa_mvp on a context holding a resident sim (home order): use another context");
  const int64_t n = c->n, nrows = c->last_re - c->last_rb;
  // staging: 6 full-N fp64 inputs + flags + per-row in/out
  const size_t need = (size_t)n * 8 * 4 + (size_t)n * 2 + (size_t)nrows * (8 * 4 + 4 * 2) + 256;
  if (!bsa::ensure(c, c->mvp_stage, need, "mvp staging")) return -1;
  char *base = (char *)c->mvp_stage.p;
  auto carve = [&](size_t bytes) {
    char *q = base;
    base += (bytes + 15) & ~size_t(15);
    return q;
  };
  double *d_gse = (double *)carve(n * 8), *d_gsn = (double *)carve(n * 8);
  double *d_sel = (double *)carve(n * 8), *d_apvs = (double *)carve(n * 8);
  uint8_t *d_nr = (uint8_t *)carve(n), *d_ro = (uint8_t *)carve(n);
  double *d_alt = (double *)carve(nrows * 8), *d_trk = (double *)carve(nrows * 8);
  double *d_tas = (double *)carve(nrows * 8), *d_vs = (double *)carve(nrows * 8);
  float *d_e = (float *)carve(nrows * 4), *d_nn = (float *)carve(nrows * 4);
  hipStream_t s = c->stream;
  BSA_HIP(c, hipMemcpyAsync(d_gse, gseast, n * 8, hipMemcpyHostToDevice, s));
  BSA_HIP(c, hipMemcpyAsync(d_gsn, gsnorth, n * 8, hipMemcpyHostToDevice, s));
  BSA_HIP(c, hipMemcpyAsync(d_sel, selalt, n * 8, hipMemcpyHostToDevice, s));
  BSA_HIP(c, hipMemcpyAsync(d_apvs, apvs, n * 8, hipMemcpyHostToDevice, s));
  if (noreso) BSA_HIP(c, hipMemcpyAsync(d_nr, noreso, n, hipMemcpyHostToDevice, s));
  if (resooff) BSA_HIP(c, hipMemcpyAsync(d_ro, resooff, n, hipMemcpyHostToDevice, s));
  BSA_HIP(c, hipMemcpyAsync(d_alt, asas_alt, nrows * 8, hipMemcpyHostToDevice, s));
  bsa::MvpDev d;
  d.gseast = d_gse;
  d.gsnorth = d_gsn;
  d.vs = (const double *)c->own[5].p;
  d.alt = (const double *)c->own[4].p;
  d.trk = (const double *)c->own[2].p;
  d.gs = (const double *)c->own[3].p;
  d.selalt = d_sel;
  d.apvs = d_apvs;
  d.aptrk = d.aptas = d.apalt = nullptr;
  d.noreso = noreso ? d_nr : nullptr;
  d.resooff = resooff ? d_ro : nullptr;
  d.asas_alt = d_alt;
  d.o_trk = d_trk;
  d.o_tas = d_tas;
  d.o_vs = d_vs;
  d.o_asase = d_e;
  d.o_asasn = d_nn;
  d.o_tsolv = nullptr;
  if (bsa::mvp_device(c, *p, d, nullptr, nullptr, nullptr, nullptr, nullptr, true)) return -1;
  BSA_HIP(c, hipMemcpyAsync(asas_alt, d_alt, nrows * 8, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipMemcpyAsync(trk, d_trk, nrows * 8, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipMemcpyAsync(tas, d_tas, nrows * 8, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipMemcpyAsync(vs, d_vs, nrows * 8, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipMemcpyAsync(asase, d_e, nrows * 4, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipMemcpyAsync(asasn, d_nn, nrows * 4, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipStreamSynchronize(s));
  return 0;
}

extern "C" int bsa_set_pairs(bsa_ctx *cc, int64_t P, const int32_t *ci, const int32_t *cj,
                             const double *qdr, const double *dist, const double *tcpa,
                             const double *tlos) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  if (P < 0) return bsa::fail(c, "negative pair count");
  if (P > 0 && (!ci || !cj || !qdr || !dist || !tcpa || !tlos)) return bsa::fail(c, "NULL pair array");
  for (int64_t k = 0; k < P; ++k) {
    if (ci[k] < 0 || ci[k] >= c->n || cj[k] < 0 || cj[k] >= c->n)
      return bsa::fail(c, "pair %lld index out of range", (long long)k);
    if (k && ci[k] < ci[k - 1]) return bsa::fail(c, "pairs not in row-major (ci non-decreasing) order");
  }
  BSA_HIP(c, hipSetDevice(c->device));
  const size_t Pn = (size_t)std::max<int64_t>(P, 1);
  if (!bsa::ensure(c, c->out_ci, Pn * 4, "ci") || !bsa::ensure(c, c->out_cj, Pn * 4, "cj") ||
      !bsa::ensure(c, c->out_pay, Pn * 5 * 8, "pair payload") ||
      !bsa::ensure(c, c->inconf, (size_t)std::max<int64_t>(c->n, 1), "inconf") ||
      !bsa::ensure(c, c->tcpamax, (size_t)std::max<int64_t>(c->n, 1) * 8, "tcpamax"))
    return -1;
  hipStream_t s = c->stream;
  double *pay = (double *)c->out_pay.p;
  if (P > 0) {
    BSA_HIP(c, hipMemcpyAsync(c->out_ci.p, ci, P * 4, hipMemcpyHostToDevice, s));
    BSA_HIP(c, hipMemcpyAsync(c->out_cj.p, cj, P * 4, hipMemcpyHostToDevice, s));
    BSA_HIP(c, hipMemcpyAsync(pay + 0 * P, qdr, P * 8, hipMemcpyHostToDevice, s));
    BSA_HIP(c, hipMemcpyAsync(pay + 1 * P, dist, P * 8, hipMemcpyHostToDevice, s));
    BSA_HIP(c, hipMemcpyAsync(pay + 2 * P, tcpa, P * 8, hipMemcpyHostToDevice, s));
    BSA_HIP(c, hipMemcpyAsync(pay + 3 * P, tlos, P * 8, hipMemcpyHostToDevice, s));
  }
  BSA_HIP(c, hipStreamSynchronize(s));
  c->last_rb = 0;
  c->last_re = c->n;
  c->last_conf = P;
  c->last_los = 0;
  c->last_flags = 0;
  c->have_pairs = true;
  return 0;
}
