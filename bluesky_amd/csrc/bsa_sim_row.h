// One row of the resident step's K4' (Pilot.APorASAS + the kinematic update +
// the next detect's record), shared by k_sim_pilot_kin (bsa_sim.hip) and K2's
// fused form (k_rank_rows<true>, bsa_cd.hip).
#pragma once
#include "bsa_kin_math.h"
#include "bsa_mvp_row.h"
#include "bsa_prep.h"

#pragma clang fp contract(off)

namespace bsa {

struct SimDev {
  double *lat, *lon, *trk, *gs, *alt, *vs, *tas, *hdg, *gse, *gsn;
  // where the step writes alt / vs / gseast / gsnorth: the same arrays, or
  // (K2's fused form) the other half of a double buffer -- K2's pairs of other
  // workgroups still read the intruders' step-start values from the first
  double *alt_w, *vs_w, *gse_w, *gsn_w;
  double *altprev;                 // pre-step altitude: the ACDATA feed derives traf.cas =
                                   // vtas2cas(tas, altprev) (traffic.py:434) off the step
  double *ax;                      // traf.ax (traffic.py:431), read by the OpenAP limits next step
  const double *env;               // OpenAP envelope, 6 x n (hmax vmin vmax vsmin vsmax axmax) or NULL
  const double *ptab;              // OpenAP type table (bsa_sim_set_perf) or NULL: envelope and
  const int *ptype;                //   acceleration follow each aircraft's flight phase
  uint8_t *phase;
  double *atm;                     // traf.p / rho / Temp (traffic.py:389), 3 x n, or NULL
  int n;
  const double *aptrk, *aptas, *apalt, *apvs, *bank, *eps, *accel;
  const double *atrk, *atas, *avs, *aalt;
  const uint8_t *active;
  const unsigned *sticky;          // abort flag of the step batch
  unsigned long long *steps_done;  // steps completed in the batch
};

struct PrepArgs {
  PrepOut out;
  TileBox *sbox, *gbox;  // (the tile boxes follow from the group boxes in the detect's K0z)
  double rpz, hpz, tla;
  int mid, rec, n;
  // tile-pair list reuse: the last build's records; a record
  // outside its budgets raises tpr_ctl[0] (the next detect rebuilds), or NULL
  const PFRec *snap;
  unsigned long long *tpr_ctl;
  float dx, ds, dv;
  unsigned long long *nf;  // non-finite tcpa inputs: the epoch stored (Ctx::nonfin), or NULL
  unsigned long long nfe;
  // HK (Ctx::hk_*): the next detect's prediction word, raised when a record
  // left pf x every budget (the list is rebuilt two detects on), or NULL
  unsigned long long *pred;
  float pf;
};

// one row of K4' (below).  The row's state is loaded before K3's part runs
// (the loads overlap; K3 writes only the ASAS targets / asas.active, which
// this lane then takes from its registers, MvpRowOut), so the row's memory
// latency is paid about once instead of along a chain of dependent accesses.
template <bool FUSE, bool PREP>
__device__ __forceinline__ PFRec pilot_kin_row(int rb, int k, double simdt, int winddim, double vwn, double vwe,
                                               const WindField &wf, const SimDev &d, const MvpIn &mv,
                                               const bsa_mvp_params &mp, const PrepArgs &pa) {
  kin::In s;
  s.tas = d.tas[k];
  s.hdg = d.hdg[k];
  s.alt = d.alt[k];
  s.vs = d.vs[k];
  s.lat = d.lat[k];
  s.lon = d.lon[k];
  s.bank = d.bank[k];
  s.eps = d.eps[k];
  s.accel = d.accel[k];
  const double aptrk = d.aptrk[k], aptas = d.aptas[k], apalt = d.apalt[k], apvs = d.apvs[k];
  double atrk = d.atrk[k], atas = d.atas[k], avs = d.avs[k], aalt = d.aalt[k];
  bool act = d.active[k] != 0;
  const double ax0 = (d.ptab || d.env) ? d.ax[k] : 0.0;
  if (FUSE) {
    const MvpRowOut o = mvp_row(rb, k - rb, mp, mv);
    if (o.act_valid) act = o.active != 0;
    if (o.valid) {
      atrk = o.trk;
      atas = o.tas;
      avs = o.vs;
      aalt = o.alt;
    }
  }
  if (winddim == 2) {  // pilot.py:32 and traffic.py:463 read the field at the same pre-step position
    kin::windfield_2d(wf, s.lat, s.lon, vwn, vwe);
    winddim = 1;
  }
  const double ptrk = act ? atrk : aptrk;             // pilot.py:41
  double asastas = atas;                              // pilot.py:37-38: no wind, GS = TAS
  if (winddim > 0) {                                  // pilot.py:31-35: ASAS GS -> TAS
    double sa, ca;
    sincos(atrk * kD2R, &sa, &ca);
    const double asastasnorth = atas * ca - vwn;
    const double asastaseast = atas * sa - vwe;
    asastas = sqrt(asastasnorth * asastasnorth + asastaseast * asastaseast);
  }
  s.ptas = act ? asastas : aptas;                     // pilot.py:42
  s.palt = act ? aalt : apalt;                        // pilot.py:43
  s.pvs = fabs(act ? avs : apvs);                     // pilot.py:44,48
  if (winddim > 0) {                                  // pilot.py:51-61: wind correction
    const double Vw = sqrt(vwn * vwn + vwe * vwe);
    const double winddir = atan2(vwe, vwn);
    const double drift = ptrk * kD2R - winddir;
    const double steer = asin(kin::npmin(1.0, kin::npmax(-1.0, Vw * sin(drift) / kin::npmax(0.001, s.tas))));
    s.phdg = kin::nprem(ptrk + steer * kR2D, 360.);
  } else {
    s.phdg = kin::nprem(ptrk, 360.);                  // pilot.py:63
  }
  if (d.atm) {  // Traffic.update's first statement: p, rho, Temp = vatmos(alt) (traffic.py:389)
    double p, rho, T;
    kin::vatmos(s.alt, p, rho, T);
    d.atm[k] = p;
    d.atm[d.n + k] = rho;
    d.atm[2 * d.n + k] = T;
  }
  if (d.ptab) {  // OpenAP.update (perfoap.py:115-131) on the pre-step state, then applylimits
    const double *row = d.ptab + (size_t)d.ptype[k] * kin::kPerfCols;
    const int ph = kin::openap_phase(row[22], s.vs, s.alt);
    d.phase[k] = (uint8_t)ph;
    kin::openap_limits(kin::openap_envelope(row, ph), ax0, s.ptas, s.pvs, s.palt);
    s.accel = ph == kin::kPhaseGD ? 2.0 : 0.5;  // OpenAP.acceleration (perfoap.py:271-280)
  } else if (d.env) {  // Pilot.applylimits (pilot.py:65-68, OpenAP), traffic.py:404
    const kin::Envelope e{d.env[k], d.env[d.n + k], d.env[2 * d.n + k], d.env[3 * d.n + k],
                          d.env[4 * d.n + k], d.env[5 * d.n + k]};
    kin::openap_limits(e, ax0, s.ptas, s.pvs, s.palt);
  }
  const kin::Out o = kin::step(s, simdt, winddim, vwn, vwe);
  d.tas[k] = o.tas;
  d.hdg[k] = o.hdg;
  d.alt_w[k] = o.alt;
  d.vs_w[k] = o.vs;
  d.lat[k] = o.lat;
  d.lon[k] = o.lon;
  d.gs[k] = o.gs;
  d.trk[k] = o.trk;
  d.gse_w[k] = o.gseast;
  d.gsn_w[k] = o.gsnorth;
  d.altprev[k] = s.alt;
  d.ax[k] = o.ax;
  if (PREP) {
    // the record's trig from the step's: sin / cos of the new latitude, and
    // without wind gs sin / cos(trk) = tas sin / cos(hdg) = gseast / gsnorth
    double trig[4] = {o.sinlat, o.coslat, o.gseast, o.gsnorth};
    if (winddim != 0) {
      double st, ct;
      sincos(o.trk * kD2R, &st, &ct);
      trig[2] = o.gs * st;
      trig[3] = o.gs * ct;
    }
    return prep_home_record(k, o.lat, o.lon, o.trk, o.gs, o.alt, o.vs, pa.rpz, pa.hpz, pa.tla, pa.mid, pa.rec, pa.out,
                            pa.nf, pa.nfe, trig);
  }
  return PFRec{};
}

// K2 fused with K4' (one rank, bsa_sim_step): the resident step's K4' run by
// k_rank_rows<true> on each workgroup's rows right after their fold, with
// alt / vs / gseast / gsnorth written to the other half of a double buffer
struct K24Args {
  SimDev d;
  MvpIn mv;           // (its gate is the workgroup's own {overflow, P} in LDS)
  bsa_mvp_params mp;
  PrepArgs pa;
  WindField wf;
  double simdt, vwn, vwe;
  int winddim, prep;
  HkPub pub;          // HK: this detect's prediction to the host (slot NULL: none)
};
int k24_launch(Ctx *c, const K24Args &ka);  // the deferred K2 launch of the last detect, fused (bsa_cd.hip)

}  // namespace bsa
