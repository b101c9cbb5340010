// K3: MVP conflict resolution on the device-resident, canonically sorted
// conflict pairs of the last detect.
//
// bluesky/traffic/asas/MVP.py:14-143 loops over confpairs and only ever
// writes dv[id1] (MVP.py:46-61; prioRules' dv2 is discarded), and confpairs
// are in row-major order, so each ownship's dv is a sequential fold over its
// own contiguous segment of pairs in j order.  One lane per ownship walks its
// segment in that order, which reproduces the reference's summation order
// exactly (no tree reduction); then the same lane runs the per-aircraft
// finalize (MVP.py:67-143).
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

__device__ __forceinline__ double np_max2(double a, double b) { return (a >= b || a != a) ? a : b; }
__device__ __forceinline__ double np_min2(double a, double b) { return (a <= b || a != a) ? a : b; }
// numpy.sign for float64
__device__ __forceinline__ double np_sign(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}
// numpy.remainder(a, b) for float64 (npy_divmod semantics)
__device__ __forceinline__ double np_rem(double a, double b) {
  double mod = fmod(a, b);
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}

// segment start of each row: first k with ci[k] >= rb + r  (ci sorted)
__global__ __launch_bounds__(256) void k_segments(int nrows, int rb, int64_t P,
                                                  const int *__restrict__ ci,
                                                  int64_t *__restrict__ seg) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > nrows) return;
  const int key = rb + r;
  int64_t lo = 0, hi = P;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (ci[mid] < key) lo = mid + 1; else hi = mid;
  }
  seg[r] = lo;
}

struct MvpIn {
  const int *cj;
  const double *qdr, *dist, *tcpa, *tlos;  // sorted pair payload
  const int64_t *seg;
  const double *gseast, *gsnorth, *vs, *alt, *trk, *gs;  // full-N traffic arrays
  const double *selalt, *apvs;                           // full-N
  const uint8_t *noreso, *resooff;                       // full-N flags or NULL
  double *asas_alt;                                      // rows [rb, re), in/out
  double *o_trk, *o_tas, *o_vs;                          // rows [rb, re)
  float *o_asase, *o_asasn;
  double *o_tsolv;                                       // optional (may be NULL)
};

__global__ __launch_bounds__(256) void k_mvp(int nrows, int rb, bsa_mvp_params p, MvpIn in) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const int id1 = rb + r;
  const double gse1 = in.gseast[id1], gsn1 = in.gsnorth[id1], vs1 = in.vs[id1], alt1 = in.alt[id1];
  double dvx = 0.0, dvy = 0.0, dvz = 0.0;
  double tsv = 1e9;  // np.ones(n) * 1e9
  const bool resooff1 = p.swresooff && in.resooff && in.resooff[id1];
  for (int64_t k = in.seg[r]; k < in.seg[r + 1]; ++k) {
    const int id2 = in.cj[k];
    const double dist = in.dist[k], tcpa = in.tcpa[k], tLOS = in.tlos[k];
    // ---- MVP.MVP (MVP.py:149-231)
    const double qdr = in.qdr[k] * kD2R;
    const double drel0 = sin(qdr) * dist;
    const double drel1 = cos(qdr) * dist;
    const double drel2 = in.alt[id2] - alt1;
    const double vrel0 = in.gseast[id2] - gse1;
    const double vrel1 = in.gsnorth[id2] - gsn1;
    const double vrel2 = in.vs[id2] - vs1;
    double dcpa0 = drel0 + vrel0 * tcpa;
    double dcpa1 = drel1 + vrel1 * tcpa;
    double dabsH = sqrt(dcpa0 * dcpa0 + dcpa1 * dcpa1);
    const double iH = p.Rm - dabsH;
    if (dabsH <= 10.) {
      dabsH = 10.;
      dcpa0 = drel1 / dist * dabsH;
      dcpa1 = -drel0 / dist * dabsH;
    }
    double dv1 = (iH * dcpa0) / (fabs(tcpa) * dabsH);
    double dv2 = (iH * dcpa1) / (fabs(tcpa) * dabsH);
    if (p.Rm < dist && dabsH < dist) {
      const double erratum = cos(asin(p.Rm / dist) - asin(dabsH / dist));
      dv1 = dv1 / erratum;
      dv2 = dv2 / erratum;
    }
    const bool vz = fabs(vrel2) > 0.0;
    double iV = vz ? p.dhm : p.dhm - fabs(drel2);
    double tsolV = vz ? fabs(drel2 / vrel2) : tLOS;
    if (tsolV > p.dtlookahead) {
      tsolV = tLOS;
      iV = p.dhm;
    }
    double dv3 = vz ? (iV / tsolV) * (-vrel2 / fabs(vrel2)) : (iV / tsolV);
    if (tsolV < tsv) tsv = tsolV;
    // ---- accumulation (MVP.py:44-61)
    if (p.swprio) {
      const double vs2 = in.vs[id2];
      const bool c1 = fabs(vs1) < 0.1 && fabs(vs2) > 0.1;  // ac1 cruising, ac2 climbing
      const bool c2 = fabs(vs2) < 0.1 && fabs(vs1) > 0.1;  // ac2 cruising, ac1 climbing
      switch (p.priocode) {
        case BSA_PRIO_FF1:
          dv3 = dv3 / 2.0;
          dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3;
          break;
        case BSA_PRIO_FF2:
          dv3 = dv3 / 2.0;
          if (!c1) { dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3; }
          break;
        case BSA_PRIO_FF3:
          if (c1) { dv3 = 0.0; dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3; }
          else if (c2) { dv3 = 0.0; }
          else { dv3 = dv3 / 2.0; dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3; }
          break;
        case BSA_PRIO_LAY1:
          dv3 = 0.0;
          if (!c1) { dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3; }
          break;
        case BSA_PRIO_LAY2:
          dv3 = 0.0;
          if (!c2) { dvx = dvx - dv1; dvy = dvy - dv2; dvz = dvz - dv3; }
          break;
        default:
          break;  // unknown code: prioRules changes nothing
      }
    } else {
      dv3 = 0.5 * dv3;
      dvx = dvx - dv1;
      dvy = dvy - dv2;
      dvz = dvz - dv3;
    }
    if (p.swnoreso && in.noreso && in.noreso[id2]) {
      dvx = dvx + dv1;
      dvy = dvy + dv2;
      dvz = dvz + dv3;
    }
    if (resooff1) dvx = dvy = dvz = 0.0;
  }

  // ---- per-aircraft finalize (MVP.py:67-143)
  const double newv0 = dvx + gse1, newv1 = dvy + gsn1, newv2 = dvz + vs1;
  const bool ids = dvx * dvx + dvy * dvy > 0;
  double newtrack, newgs, newvs;
  const double trk1 = in.trk[id1], gs1 = in.gs[id1];
  if (p.swresohoriz) {
    if (p.swresospd && !p.swresohdg) {
      newtrack = trk1;
      newgs = sqrt(newv0 * newv0 + newv1 * newv1);
      newvs = vs1;
    } else if (p.swresohdg && !p.swresospd) {
      newtrack = np_rem(atan2(newv0, newv1) * 180 / kPI, 360);
      newgs = gs1;
      newvs = vs1;
    } else {
      newtrack = np_rem(atan2(newv0, newv1) * 180 / kPI, 360);
      newgs = sqrt(newv0 * newv0 + newv1 * newv1);
      newvs = vs1;
    }
  } else if (p.swresovert) {
    newtrack = trk1;
    newgs = gs1;
    newvs = newv2;
  } else {
    newtrack = np_rem(atan2(newv0, newv1) * 180 / kPI, 360);
    newgs = sqrt(newv0 * newv0 + newv1 * newv1);
    newvs = newv2;
  }
  const double tas = np_max2(p.vmin, np_min2(p.vmax, newgs));
  const double vsc = np_max2(p.vsmin, np_min2(p.vsmax, newvs));
  in.o_trk[r] = newtrack;
  in.o_tas[r] = tas;
  in.o_vs[r] = vsc;
  in.o_asase[r] = ids ? (float)(tas * sin(newtrack / 180 * kPI)) : 0.0f;
  in.o_asasn[r] = ids ? (float)(tas * cos(newtrack / 180 * kPI)) : 0.0f;

  const double selalt = in.selalt[id1];
  double aalt = in.asas_alt[r];
  const double signdvs = np_sign(vsc - in.apvs[id1] * np_sign(selalt - alt1));
  const double signalt = np_sign(aalt - selalt);
  aalt = (signdvs == 0 || signdvs == signalt) ? aalt : selalt;
  if (tsv < p.dtlookahead && fabs(dvz) > 0.0) aalt = vsc * tsv + alt1;
  const double hz = p.swresohoriz ? 1.0 : 0.0;
  in.asas_alt[r] = aalt * (1.0 - hz) + selalt * hz;
  if (in.o_tsolv) in.o_tsolv[r] = tsv;
}

// Device-side MVP over the last detect's pairs; all pointers are device
// pointers (full-N traffic arrays, per-row outputs).
int mvp_device(Ctx *c, const bsa_mvp_params &p, const MvpDev &d) {
  if (!c->have_pairs) return fail(c, "bsa_mvp: no detect results (call bsa_detect first)");
  const int64_t rb = c->last_rb, re = c->last_re, nrows = re - rb, P = c->last_conf;
  if (nrows <= 0) return 0;
  if (!ensure(c, c->seg, (size_t)(nrows + 1) * 8, "mvp segments")) return -1;
  hipLaunchKernelGGL(k_segments, dim3((unsigned)((nrows + 1 + 255) / 256)), dim3(256), 0, c->stream,
                     (int)nrows, (int)rb, P, (const int *)c->out_ci.p, (int64_t *)c->seg.p);
  BSA_HIP(c, hipGetLastError());
  const double *pay = (const double *)c->out_pay.p;
  MvpIn in;
  in.cj = (const int *)c->out_cj.p;
  in.qdr = pay + 0 * P;
  in.dist = pay + 1 * P;
  in.tcpa = pay + 2 * P;
  in.tlos = pay + 3 * P;
  in.seg = (const int64_t *)c->seg.p;
  in.gseast = d.gseast;
  in.gsnorth = d.gsnorth;
  in.vs = d.vs;
  in.alt = d.alt;
  in.trk = d.trk;
  in.gs = d.gs;
  in.selalt = d.selalt;
  in.apvs = d.apvs;
  in.noreso = d.noreso;
  in.resooff = d.resooff;
  in.asas_alt = d.asas_alt;
  in.o_trk = d.o_trk;
  in.o_tas = d.o_tas;
  in.o_vs = d.o_vs;
  in.o_asase = d.o_asase;
  in.o_asasn = d.o_asasn;
  in.o_tsolv = d.o_tsolv;
  hipLaunchKernelGGL(k_mvp, dim3((unsigned)((nrows + 255) / 256)), dim3(256), 0, c->stream,
                     (int)nrows, (int)rb, p, in);
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
  d.noreso = noreso ? d_nr : nullptr;
  d.resooff = resooff ? d_ro : nullptr;
  d.asas_alt = d_alt;
  d.o_trk = d_trk;
  d.o_tas = d_tas;
  d.o_vs = d_vs;
  d.o_asase = d_e;
  d.o_asasn = d_nn;
  d.o_tsolv = nullptr;
  if (bsa::mvp_device(c, *p, d)) return -1;
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
