// Device-side math of one aircraft's kinematic step, shared by the host-API
// kernel (bsa_kin.hip) and the GPU-resident sim step (bsa_sim.hip).
//
// Traffic.UpdateAirSpeed    bluesky/traffic/traffic.py:425-454
// Traffic.UpdateGroundSpeed bluesky/traffic/traffic.py:456-476 (winddim 0/1/2)
// Windfield.getdata, 2-D    bluesky/traffic/windfield.py:158-179 (winddim 2)
// Traffic.UpdatePosition    bluesky/traffic/traffic.py:478-483
// aero.vatmos / vtas2cas / vtas2mach  bluesky/tools/aero.py:62-147
// Every expression keeps numpy's evaluation order (compile with
// -ffp-contract=off).
#pragma once
#include "bsa_geo_math.h"
#include "bsa_internal.h"

namespace bsa {

// 2-D wind field (winddim 2): nvec definition points with their wind
// (Windfield.lat / lon / vnorth[0, :] / veast[0, :]), device pointers.
struct WindField {
  const double *lat, *lon, *vn, *ve;
  int nvec;
};

namespace kin {

// Windfield.getdata for a 2-D field at one position (windfield.py:158-179):
// inverse-distance-squared weights in a flat frame of 1-degree units,
// normalised by their sum.  The reference's sums are BLAS dot products; here
// they run in point order (same terms, summation order may differ by ulps).
__device__ __forceinline__ void windfield_2d(const WindField &w, double lat, double lon, double &vn,
                                             double &ve) {
  const double eps = 1e-20;
  double sum = 0.0;
  for (int k = 0; k < w.nvec; ++k) {
    const double cavelat = cos((0.5 * (lat + w.lat[k])) * kD2R);
    const double dy = lat - w.lat[k];
    const double dx = cavelat * (lon - w.lon[k]);
    sum += 1. / (eps + dx * dx + dy * dy);
  }
  vn = 0.0;
  ve = 0.0;
  for (int k = 0; k < w.nvec; ++k) {
    const double cavelat = cos((0.5 * (lat + w.lat[k])) * kD2R);
    const double dy = lat - w.lat[k];
    const double dx = cavelat * (lon - w.lon[k]);
    const double horfact = (1. / (eps + dx * dx + dy * dy)) / sum;
    vn += w.vn[k] * horfact;
    ve += w.ve[k] * horfact;
  }
}

constexpr double kG0 = 9.80665;        // aero.py:18
constexpr double kRgas = 287.05287;    // aero.py:19
constexpr double kP0 = 101325.;        // aero.py:20
constexpr double kRho0 = 1.225;        // aero.py:21
constexpr double kTstrat = 216.65;     // aero.py:23
constexpr double kGamma = 1.40;        // aero.py:24
constexpr double kRearth = 6371000.;   // aero.py:28
constexpr double kFPM = kFT / 60.;     // aero.py:13

__device__ __forceinline__ double npmax(double a, double b) { return (a >= b || a != a) ? a : b; }
__device__ __forceinline__ double npmin(double a, double b) { return (a <= b || a != a) ? a : b; }
__device__ __forceinline__ double npsign(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}
// numpy.remainder for float64 (npy_divmod semantics)
__device__ __forceinline__ double nprem(double a, double b) {
  double mod = b == 360.0 ? fmod360(a) : fmod(a, b);
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}

// vatmos (aero.py:62-74): pressure and density at altitude h [m]
__device__ __forceinline__ void vatmos(double h, double &p, double &rho, double &T) {
  T = npmax(288.15 - 0.0065 * h, kTstrat);
  const double rhotrop = 1.225 * pow(T / 288.15, 4.256848030018761);
  const double dhstrat = npmax(0., h - 11000.);
  rho = rhotrop * exp(-dhstrat / 6341.552161);
  p = rho * kRgas * T;
}

// aero.py:139-147 vtas2cas, aero.py:128-136 vcas2tas
__device__ __forceinline__ double vtas2cas(double tas, double h) {
  double p, rho, T;
  vatmos(h, p, rho, T);
  const double qdyn = p * (pow(1. + rho * tas * tas / (7. * p), 3.5) - 1.);
  const double cas = sqrt(7. * kP0 / kRho0 * (pow(qdyn / kP0 + 1., 2. / 7.) - 1.));
  return tas < 0 ? -1 * cas : cas;
}
__device__ __forceinline__ double vcas2tas(double cas, double h) {
  double p, rho, T;
  vatmos(h, p, rho, T);
  const double qdyn = kP0 * (pow(1. + kRho0 * cas * cas / (7. * kP0), 3.5) - 1.);
  const double tas = sqrt(7. * p / rho * (pow(1. + qdyn / p, 2. / 7.) - 1.));
  return cas < 0 ? -1 * tas : tas;
}

// per-aircraft OpenAP flight envelope (perfoap.py:185-209; vmin / vmax are CAS)
struct Envelope {
  double hmax, vmin, vmax, vsmin, vsmax, axmax;
};

// OpenAP.limits as Pilot.applylimits applies it (pilot.py:65-68) to the
// pilot's tas / vs / alt; ax = traf.ax of the previous step.
__device__ __forceinline__ void openap_limits(const Envelope &e, double ax, double &tas, double &vs,
                                              double &h) {
  const double allow_h = h > e.hmax ? e.hmax : h;
  const double intent_v_cas = vtas2cas(tas, allow_h);
  double allow_v_cas = intent_v_cas < e.vmin ? e.vmin : intent_v_cas;
  allow_v_cas = intent_v_cas > e.vmax ? e.vmax : allow_v_cas;
  const double allow_v_tas = vcas2tas(allow_v_cas, allow_h);
  const double vs_max_with_acc = (1 - ax / e.axmax) * e.vsmax;
  double allow_vs = vs > e.vsmax ? vs_max_with_acc : vs;
  allow_vs = vs < e.vsmin ? e.vsmin : allow_vs;
  tas = allow_v_tas;
  vs = allow_vs;
  h = allow_h;
}

// OpenAP type table (bsa_sim_set_perf, bluesky_amd/perf.py): per type, vmin by
// phase NA..GD, vmax by phase, vsmin, vsmax, hmax, axmax, lifttype, pad
constexpr int kPerfCols = 24;
constexpr int kPhaseGD = 8;

// OpenAP flight phase (phase.py:14-62, unit SI): the fixed-wing rule on the
// pre-step state, rotors (and any other lift type) NA
__device__ __forceinline__ int openap_phase(double lift, double vs, double alt) {
  if (lift != 1.0) return 0;
  const double roc = vs / 0.00508, a = alt / 0.3048;
  int ph = 0;
  if (a <= 10 && roc <= 100 && roc >= -100) ph = kPhaseGD;
  if (a >= 0 && a <= 1000 && roc >= 0) ph = 2;     // IC
  if (a >= 0 && a <= 1000 && roc <= 0) ph = 6;     // AP
  if (a >= 1000 && roc >= 100) ph = 3;             // CL
  if (a >= 1000 && roc <= -100) ph = 5;            // DE
  if (a >= 5000 && roc <= 100 && roc >= -100) ph = 4;  // CR
  return ph;
}

// __construct_limit_matrix (perfoap.py:211-262) for one aircraft: its type
// row at its phase
__device__ __forceinline__ Envelope openap_envelope(const double *row, int ph) {
  return Envelope{row[20], row[ph], row[9 + ph], row[18], row[19], row[21]};
}

struct In {
  double tas, hdg, alt, vs, lat, lon;       // state before the step
  double ptas, phdg, palt, pvs;             // pilot targets
  double bank, eps, accel;
};
struct Out {
  double tas, hdg, alt, vs, lat, lon;       // state after the step
  double ax, delspd, cas, mach, gsnorth, gseast, gs, trk, coslat, az;
  double sinlat;  // sin(radians(lat)) of the new position (the next records reuse it)
  bool swhdgsel, swaltsel;
};

__device__ __forceinline__ Out step(const In &s, double simdt, int winddim, double wn, double we) {
  Out o;
  // ---- UpdateAirSpeed: speed (traffic.py:427-435)
  const double delta_spd = s.ptas - s.tas;
  const double need_ax = fabs(delta_spd) > kKTS ? 1.0 : 0.0;
  o.ax = need_ax * npsign(delta_spd) * s.accel;
  o.delspd = delta_spd;
  const double tas = s.tas + o.ax * simdt;
  // vatmos(alt) (aero.py:62-74), shared by vtas2cas and vtas2mach
  double p, rho, T;
  vatmos(s.alt, p, rho, T);
  const double qdyn = p * (pow(1. + rho * tas * tas / (7. * p), 3.5) - 1.);
  double cas = sqrt(7. * kP0 / kRho0 * (pow(qdyn / kP0 + 1., 2. / 7.) - 1.));
  o.cas = tas < 0 ? -1 * cas : cas;
  o.mach = tas / sqrt(kGamma * kRgas * T);
  // turning (traffic.py:438-444)
  const double turnrate = (kG0 * tan(s.bank) / npmax(tas, s.eps)) * kR2D;
  const double delhdg = nprem(s.phdg - s.hdg + 180, 360) - 180;
  o.swhdgsel = fabs(delhdg) > fabs(2 * simdt * turnrate);
  const double hdg = nprem(s.hdg + simdt * turnrate * (o.swhdgsel ? 1.0 : 0.0) * npsign(delhdg), 360.);
  // vertical speed (traffic.py:447-454)
  const double delta_alt = s.palt - s.alt;
  o.swaltsel = fabs(delta_alt) > npmax(10 * kFT, fabs(2 * simdt * fabs(s.vs)));
  const double target_vs = (o.swaltsel ? 1.0 : 0.0) * npsign(delta_alt) * fabs(s.pvs);
  const double delta_vs = target_vs - s.vs;
  const bool need_az = fabs(delta_vs) > 300 * kFPM;
  o.az = (need_az ? 1.0 : 0.0) * npsign(delta_vs) * (300 * kFPM);
  double vs = need_az ? s.vs + o.az * simdt : target_vs;
  vs = isfinite(vs) ? vs : 0;

  // ---- UpdateGroundSpeed (traffic.py:456-476)
  double sh, ch;
  sincos(hdg * kD2R, &sh, &ch);
  if (winddim == 0) {
    o.gsnorth = tas * ch;
    o.gseast = tas * sh;
    o.gs = tas;
    o.trk = hdg;
  } else {
    const double aw = s.alt > 50. * kFT ? 1.0 : 0.0;
    const double naw = 1.0 - aw;
    o.gsnorth = tas * ch + wn * aw;
    o.gseast = tas * sh + we * aw;
    o.gs = naw * tas + aw * sqrt(o.gsnorth * o.gsnorth + o.gseast * o.gseast);
    o.trk = naw * hdg + nprem(aw * (atan2(o.gseast, o.gsnorth) * kR2D), 360.);
  }

  // ---- UpdatePosition (traffic.py:480-483)
  o.alt = o.swaltsel ? s.alt + vs * simdt : s.palt;
  o.lat = s.lat + (simdt * o.gsnorth / kRearth) * kR2D;
  sincos(o.lat * kD2R, &o.sinlat, &o.coslat);
  o.lon = s.lon + (simdt * o.gseast / o.coslat / kRearth) * kR2D;
  o.tas = tas;
  o.hdg = hdg;
  o.vs = vs;
  return o;
}

}  // namespace kin
}  // namespace bsa
