// K3's per-row part (MVP.py:44-143), shared by k_mvp_row (bsa_mvp.hip) and
// the resident step's fused MVP + pilot + kinematics kernel (bsa_sim.hip).
#pragma once
#include "bsa_geo_math.h"  // np_max / np_min / np_rem
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

// numpy.sign for float64
__device__ __forceinline__ double np_sign(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}
struct MvpIn {
  const int *ci, *cj;
  const double *pay;                 // sorted pair payload, 5 x P (qdr dist tcpa tlos dcpa)
  const unsigned *seg;               // row segments, nrows + 1 entries; seg[nrows] = P
  const double *gseast, *gsnorth, *vs, *alt, *trk, *gs;  // full-N traffic arrays
  const double *selalt, *apvs;                           // full-N
  const double *aptrk, *aptas, *apalt;                   // full-N, resident CR OFF only (else NULL)
  const uint8_t *noreso, *resooff;                       // full-N flags or NULL
  double *asas_alt;                                      // rows [rb, re), in/out
  double *o_trk, *o_tas, *o_vs;                          // rows [rb, re)
  float *o_asase, *o_asasn;
  double *o_tsolv;                                       // optional (may be NULL)
  double4 *pdv;                                          // per pair: dv1 dv2 dv3 tsolV
  uint8_t *pfl;                                          // per pair: bit0 subtract, bit1 add back
  // per row, or NULL: the fold below already done by K2 (k_rank_rows, the
  // same operations in the same order): dv1 dv2 dv3 min tsolV
  const double4 *rowdv;
  // resident sim step only (else NULL): gate = {overflow, P (max over ranks)},
  // sticky = abort flag of the whole step batch, inconf -> active copy
  const unsigned long long *gate;
  unsigned *sticky;
  const uint8_t *inconf;
  uint8_t *active;
  int nrows;
  int resolve;                                           // 0: CR OFF (DoNothing.py), resident step only
  // rows [rb, re) or NULL: NaN when the (all-reduced) gate says some rank's
  // columns hold a non-finite tcpa input (several ranks: K2 knew its own only)
  unsigned long long *tcpamax;
};

__device__ __forceinline__ bool mvp_aborted(const MvpIn &in) {
  return in.gate && (in.sticky[0] != 0 || in.gate[0] >= kGateOverflow);
}

// The dv fold of one row over its pairs in confpair order (MVP.py:44-61):
// dv -= dv_mvp (and += again for the prioRules / noreso cases, the flags of
// the pair), timesolveV = the minimum tsolV.  resooff is applied by the
// caller (MVP.py:58-59 zeroes dv inside the loop: the same as zeroing the
// result, a row without pairs keeps +0).  Loads of 4 pairs are issued
// together (a row's pairs are contiguous).
__device__ __forceinline__ double4 mvp_fold(const double4 *__restrict__ pdv, const uint8_t *__restrict__ pfl,
                                            unsigned b, unsigned e) {
  double dvx = 0.0, dvy = 0.0, dvz = 0.0;
  double tsv = 1e9;  // np.ones(n) * 1e9
  for (unsigned k0 = b; k0 < e; k0 += 4) {
    double4 d[4];
    uint8_t f[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const unsigned k = k0 + u < e ? k0 + u : b;
      d[u] = pdv[k];
      f[u] = pfl[k];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u >= e) break;
      if (d[u].w < tsv) tsv = d[u].w;
      if (f[u] & 1) {
        dvx = dvx - d[u].x;
        dvy = dvy - d[u].y;
        dvz = dvz - d[u].z;
      }
      if (f[u] & 2) {
        dvx = dvx + d[u].x;
        dvy = dvy + d[u].y;
        dvz = dvz + d[u].z;
      }
    }
  }
  return make_double4(dvx, dvy, dvz, tsv);
}

// the row's new ASAS targets (valid: MVP or DoNothing wrote them this call)
// and asas.active (act_valid: copied from inconf), for a caller that goes on
// with them in registers (the resident step's pilot, K4')
struct MvpRowOut {
  bool valid, act_valid;
  uint8_t active;
  double trk, tas, vs, alt;
};

// Per row: the dv fold over the row's pairs in confpair order (MVP.py:44-61),
// then the per-aircraft finalize (MVP.py:67-143).  In the resident sim step
// this kernel also gates the step (overflow -> sticky abort), copies
// asas.active = inconf (the stand-in for ResumeNav without resume_nav) and,
// with CR OFF, runs DoNothing.resolve instead of MVP.  Every load of the row
// is issued first (the stores go to other arrays or to this row's own
// words), so their latencies overlap instead of forming a chain.
__device__ __forceinline__ MvpRowOut mvp_row(int rb, int r, const bsa_mvp_params &p, const MvpIn &in) {
  MvpRowOut res{false, false, 0, 0.0, 0.0, 0.0, 0.0};
  const int id1 = rb + r;
  const uint8_t inc = in.gate && in.inconf ? in.inconf[r] : 0;
  const unsigned long long P = in.gate ? in.gate[1] : 1ull;
  const double gse1 = in.gseast[id1], gsn1 = in.gsnorth[id1], vs1 = in.vs[id1], alt1 = in.alt[id1];
  const double trk1 = in.trk[id1], gs1 = in.gs[id1];
  const double selalt = in.selalt[id1], apvs1 = in.apvs[id1];
  const double aalt0 = in.asas_alt[r];
  const bool resooff1 = p.swresooff && in.resooff && in.resooff[id1];
  double4 fold = make_double4(0.0, 0.0, 0.0, 1e9);
  unsigned s0 = 0, s1 = 0;
  if (in.rowdv) fold = in.rowdv[r];
  else {
    s0 = in.seg[r];
    s1 = in.seg[r + 1];
  }
  const bool nothing = in.gate && !in.resolve;
  double aptrk1 = 0.0, aptas1 = 0.0, apalt1 = 0.0;
  if (nothing) {
    aptrk1 = in.aptrk[id1];
    aptas1 = in.aptas[id1];
    apalt1 = in.apalt[id1];
  }
  if (in.gate) {
    if (in.tcpamax && in.gate[0] == kGateNonfinite) in.tcpamax[r] = kNanBits;  // (StateBasedCD.py:90)
    if (in.inconf) {  // stand-in for ResumeNav unless resume_nav
      in.active[id1] = inc;
      res.act_valid = true;
      res.active = inc;
    }
    // asas.py:486-487: resolve only if confpairs is non-empty (over all ranks)
    if (P == 0) return res;
    if (nothing) {  // CR "OFF" = DoNothing.resolve (DoNothing.py:11-20, asas.py:41,76-77):
      in.o_trk[r] = aptrk1;  // the ASAS targets become the autopilot's
      in.o_tas[r] = aptas1;
      in.o_vs[r] = apvs1;
      in.asas_alt[r] = apalt1;
      res.valid = true;
      res.trk = aptrk1;
      res.tas = aptas1;
      res.vs = apvs1;
      res.alt = apalt1;
      return res;
    }
  }
  if (!in.rowdv) fold = mvp_fold(in.pdv, in.pfl, s0, s1);
  double dvx = fold.x, dvy = fold.y, dvz = fold.z;
  const double tsv = fold.w;
  if (resooff1) dvx = dvy = dvz = 0.0;

  // ---- per-aircraft finalize (MVP.py:67-143)
  const double newv0 = dvx + gse1, newv1 = dvy + gsn1, newv2 = dvz + vs1;
  const bool ids = dvx * dvx + dvy * dvy > 0;
  double newtrack, newgs, newvs;
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
  const double tas = np_max(p.vmin, np_min(p.vmax, newgs));
  const double vsc = np_max(p.vsmin, np_min(p.vsmax, newvs));
  in.o_trk[r] = newtrack;
  in.o_tas[r] = tas;
  in.o_vs[r] = vsc;
  double snt, cnt;
  sincos(newtrack / 180 * kPI, &snt, &cnt);
  in.o_asase[r] = ids ? (float)(tas * snt) : 0.0f;
  in.o_asasn[r] = ids ? (float)(tas * cnt) : 0.0f;

  double aalt = aalt0;
  const double signdvs = np_sign(vsc - apvs1 * np_sign(selalt - alt1));
  const double signalt = np_sign(aalt - selalt);
  aalt = (signdvs == 0 || signdvs == signalt) ? aalt : selalt;
  if (tsv < p.dtlookahead && fabs(dvz) > 0.0) aalt = vsc * tsv + alt1;
  const double hz = p.swresohoriz ? 1.0 : 0.0;
  const double aalt_out = aalt * (1.0 - hz) + selalt * hz;
  in.asas_alt[r] = aalt_out;
  if (in.o_tsolv) in.o_tsolv[r] = tsv;
  res.valid = true;
  res.trk = newtrack;
  res.tas = tas;
  res.vs = vsc;
  res.alt = aalt_out;
  return res;
}

}  // namespace bsa
