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
  // resident sim step only (else NULL): gate = {overflow, P (max over ranks)},
  // sticky = abort flag of the whole step batch, inconf -> active copy
  const unsigned long long *gate;
  unsigned *sticky;
  const uint8_t *inconf;
  uint8_t *active;
  int nrows;
  int resolve;                                           // 0: CR OFF (DoNothing.py), resident step only
};

__device__ __forceinline__ bool mvp_aborted(const MvpIn &in) {
  return in.gate && (in.sticky[0] != 0 || in.gate[0] != 0);
}

// Per row: the dv fold over the row's pairs in confpair order (MVP.py:44-61),
// then the per-aircraft finalize (MVP.py:67-143).  In the resident sim step
// this kernel also gates the step (overflow -> sticky abort), copies
// asas.active = inconf (the stand-in for ResumeNav without resume_nav) and,
// with CR OFF, runs DoNothing.resolve instead of MVP.
__device__ __forceinline__ void mvp_row(int rb, int r, const bsa_mvp_params &p, const MvpIn &in) {
  if (in.gate) {
    if (in.inconf) in.active[rb + r] = in.inconf[r];  // stand-in for ResumeNav unless resume_nav
    // asas.py:486-487: resolve only if confpairs is non-empty (over all ranks)
    if (in.gate[1] == 0) return;
    if (!in.resolve) {  // CR "OFF" = DoNothing.resolve (DoNothing.py:11-20, asas.py:41,76-77):
      const int id1 = rb + r;  // the ASAS targets become the autopilot's
      in.o_trk[r] = in.aptrk[id1];
      in.o_tas[r] = in.aptas[id1];
      in.o_vs[r] = in.apvs[id1];
      in.asas_alt[r] = in.apalt[id1];
      return;
    }
  }
  const int id1 = rb + r;
  const double gse1 = in.gseast[id1], gsn1 = in.gsnorth[id1], vs1 = in.vs[id1], alt1 = in.alt[id1];
  double dvx = 0.0, dvy = 0.0, dvz = 0.0;
  double tsv = 1e9;  // np.ones(n) * 1e9
  const bool resooff1 = p.swresooff && in.resooff && in.resooff[id1];
  const unsigned e = in.seg[r + 1];
  for (unsigned k = in.seg[r]; k < e; ++k) {
    const double4 d = in.pdv[k];
    const uint8_t f = in.pfl[k];
    if (d.w < tsv) tsv = d.w;
    if (f & 1) {
      dvx = dvx - d.x;
      dvy = dvy - d.y;
      dvz = dvz - d.z;
    }
    if (f & 2) {
      dvx = dvx + d.x;
      dvy = dvy + d.y;
      dvz = dvz + d.z;
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
  const double tas = np_max(p.vmin, np_min(p.vmax, newgs));
  const double vsc = np_max(p.vsmin, np_min(p.vsmax, newvs));
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

}  // namespace bsa
