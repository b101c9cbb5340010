// Per-pair part of MVP.resolve (MVP.py:33-56): MVP.MVP (MVP.py:149-231) and
// the priority rules (MVP.py:235-300; only the first return value is kept,
// MVP.py:46).  Shared by k_mvp_pair (bsa_mvp.hip) and the resident step's
// K2 (k_rank, bsa_cd.hip), which evaluates it as it places each pair.
#pragma once
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

// full-N traffic arrays the per-pair vector reads
struct MvpPairIn {
  const double *gseast, *gsnorth, *vs, *alt;
  const uint8_t *noreso;  // NULL = empty NORESO list
  const unsigned *id2h;   // resident step (home order): the intruder's home position; NULL = identity
};

// dv = (dv1, dv2, dv3, tsolV); fl: bit 0 subtract from dv[id1], bit 1 add back (NORESO).
// id1 indexes the arrays; id2 is the intruder's aircraft index (mapped by id2h)
__device__ __forceinline__ void mvp_pair(const bsa_mvp_params &p, const MvpPairIn &in, int id1, int id2,
                                         double qdr_deg, double dist, double tcpa, double tLOS, double4 &dv,
                                         uint8_t &fl) {
  if (in.id2h) id2 = (int)in.id2h[id2];
  const double gse1 = in.gseast[id1], gsn1 = in.gsnorth[id1], vs1 = in.vs[id1], alt1 = in.alt[id1];
  // ---- MVP.MVP (MVP.py:149-231)
  const double qdr = qdr_deg * kD2R;
  double sq, cq;
  sincos(qdr, &sq, &cq);
  const double drel0 = sq * dist;
  const double drel1 = cq * dist;
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
  // ---- accumulation rule (MVP.py:44-56): subtract? (then) add back?
  bool sub = true;
  if (p.swprio) {
    const double vs2 = in.vs[id2];
    const bool c1 = fabs(vs1) < 0.1 && fabs(vs2) > 0.1;  // ac1 cruising, ac2 climbing
    const bool c2 = fabs(vs2) < 0.1 && fabs(vs1) > 0.1;  // ac2 cruising, ac1 climbing
    switch (p.priocode) {
      case BSA_PRIO_FF1: dv3 = dv3 / 2.0; break;
      case BSA_PRIO_FF2: dv3 = dv3 / 2.0; sub = !c1; break;
      case BSA_PRIO_FF3:
        if (c1) dv3 = 0.0;
        else if (c2) { dv3 = 0.0; sub = false; }
        else dv3 = dv3 / 2.0;
        break;
      case BSA_PRIO_LAY1: dv3 = 0.0; sub = !c1; break;
      case BSA_PRIO_LAY2: dv3 = 0.0; sub = !c2; break;
      default: sub = false; break;  // unknown code: prioRules changes nothing
    }
  } else {
    dv3 = 0.5 * dv3;
  }
  const bool add = p.swnoreso && in.noreso && in.noreso[id2];
  dv = make_double4(dv1, dv2, dv3, tsolV);
  fl = (uint8_t)((sub ? 1 : 0) | (add ? 2 : 0));
}

}  // namespace bsa
