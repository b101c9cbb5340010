// K4: fused kinematic integration of one sim step, one lane per aircraft.
//
// Traffic.UpdateAirSpeed   bluesky/traffic/traffic.py:425-454
// Traffic.UpdateGroundSpeed bluesky/traffic/traffic.py:456-476 (winddim 0/1)
// Traffic.UpdatePosition   bluesky/traffic/traffic.py:478-483
// with aero.vatmos / vtas2cas / vtas2mach (bluesky/tools/aero.py:62-147)
// inlined.  HBM-bound: 13 fp64 reads + 16 fp64 + 2 byte writes per aircraft
// (234 B); every expression keeps numpy's evaluation order.
#include "bsa_internal.h"

#pragma clang fp contract(off)

namespace bsa {

namespace {
constexpr double kG0 = 9.80665;        // aero.py:18
constexpr double kRgas = 287.05287;    // aero.py:19
constexpr double kP0 = 101325.;        // aero.py:20
constexpr double kRho0 = 1.225;        // aero.py:21
constexpr double kTstrat = 216.65;     // aero.py:23
constexpr double kGamma = 1.40;        // aero.py:24
constexpr double kRearth = 6371000.;   // aero.py:28
constexpr double kFPM = kFT / 60.;     // aero.py:13

__device__ __forceinline__ double npmax(double a, double b) { return (a >= b || a != a) ? a : b; }
__device__ __forceinline__ double npsign(double x) {
  return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}
__device__ __forceinline__ double nprem(double a, double b) {
  double mod = fmod(a, b);
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}
}  // namespace

__global__ __launch_bounds__(256) void k_kinematics(int n, double simdt, int winddim, double wn,
                                                    double we, KinDev d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double tas0 = d.tas[k], hdg0 = d.hdg[k], alt0 = d.alt[k], vs0 = d.vs[k];
  const double ptas = d.ptas[k], phdg = d.phdg[k], palt = d.palt[k], pvs = d.pvs[k];

  // ---- UpdateAirSpeed: speed
  const double delta_spd = ptas - tas0;
  const double need_ax = fabs(delta_spd) > kKTS ? 1.0 : 0.0;
  const double ax = need_ax * npsign(delta_spd) * d.accel[k];
  const double tas = tas0 + ax * simdt;
  // vatmos(alt) (aero.py:62-74) shared by vtas2cas and vtas2mach
  const double T = npmax(288.15 - 0.0065 * alt0, kTstrat);
  const double rhotrop = 1.225 * pow(T / 288.15, 4.256848030018761);
  const double dhstrat = npmax(0., alt0 - 11000.);
  const double rho = rhotrop * exp(-dhstrat / 6341.552161);
  const double p = rho * kRgas * T;
  const double qdyn = p * (pow(1. + rho * tas * tas / (7. * p), 3.5) - 1.);
  double cas = sqrt(7. * kP0 / kRho0 * (pow(qdyn / kP0 + 1., 2. / 7.) - 1.));
  cas = tas < 0 ? -1 * cas : cas;
  const double a = sqrt(kGamma * kRgas * T);
  const double mach = tas / a;
  // turning
  const double turnrate = (kG0 * tan(d.bank[k]) / npmax(tas, d.eps[k])) * kR2D;
  const double delhdg = nprem(phdg - hdg0 + 180, 360) - 180;
  const bool swhdgsel = fabs(delhdg) > fabs(2 * simdt * turnrate);
  const double hdg = nprem(hdg0 + simdt * turnrate * (swhdgsel ? 1.0 : 0.0) * npsign(delhdg), 360.);
  // vertical speed
  const double delta_alt = palt - alt0;
  const bool swaltsel = fabs(delta_alt) > npmax(10 * kFT, fabs(2 * simdt * fabs(vs0)));
  const double target_vs = (swaltsel ? 1.0 : 0.0) * npsign(delta_alt) * fabs(pvs);
  const double delta_vs = target_vs - vs0;
  const bool need_az = fabs(delta_vs) > 300 * kFPM;
  const double az = (need_az ? 1.0 : 0.0) * npsign(delta_vs) * (300 * kFPM);
  double vs = need_az ? vs0 + az * simdt : target_vs;
  vs = isfinite(vs) ? vs : 0;

  // ---- UpdateGroundSpeed
  double gsnorth, gseast, gs, trk;
  if (winddim == 0) {
    gsnorth = tas * cos(hdg * kD2R);
    gseast = tas * sin(hdg * kD2R);
    gs = tas;
    trk = hdg;
  } else {
    const double aw = alt0 > 50. * kFT ? 1.0 : 0.0;
    const double naw = 1.0 - aw;
    gsnorth = tas * cos(hdg * kD2R) + wn * aw;
    gseast = tas * sin(hdg * kD2R) + we * aw;
    gs = naw * tas + aw * sqrt(gsnorth * gsnorth + gseast * gseast);
    trk = naw * hdg + nprem(aw * (atan2(gseast, gsnorth) * kR2D), 360.);
  }

  // ---- UpdatePosition
  const double alt = swaltsel ? alt0 + vs * simdt : palt;
  const double lat = d.lat[k] + (simdt * gsnorth / kRearth) * kR2D;
  const double coslat = cos(lat * kD2R);
  const double lon = d.lon[k] + (simdt * gseast / coslat / kRearth) * kR2D;

  d.tas[k] = tas;
  d.hdg[k] = hdg;
  d.alt[k] = alt;
  d.vs[k] = vs;
  d.lat[k] = lat;
  d.lon[k] = lon;
  if (d.ax) d.ax[k] = ax;
  if (d.delspd) d.delspd[k] = delta_spd;
  if (d.cas) d.cas[k] = cas;
  if (d.mach) d.mach[k] = mach;
  if (d.gsnorth) d.gsnorth[k] = gsnorth;
  if (d.gseast) d.gseast[k] = gseast;
  if (d.gs) d.gs[k] = gs;
  if (d.trk) d.trk[k] = trk;
  if (d.coslat) d.coslat[k] = coslat;
  if (d.az) d.az[k] = az;
  if (d.swhdgsel) d.swhdgsel[k] = swhdgsel;
  if (d.swaltsel) d.swaltsel[k] = swaltsel;
}

int kin_device(Ctx *c, int64_t n, double simdt, int winddim, double vn, double ve, const KinDev &d) {
  if (n <= 0) return 0;
  if (winddim != 0 && winddim != 1) return fail(c, "winddim %d not supported (0 or 1)", winddim);
  hipLaunchKernelGGL(k_kinematics, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n,
                     simdt, winddim, vn, ve, d);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

}  // namespace bsa

extern "C" int bsa_kinematics(bsa_ctx *cc, int64_t n, double simdt, int winddim, double windnorth,
                              double windeast, bsa_kin_io *io) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  if (!io) return bsa::fail(c, "NULL io");
  if (n < 0 || n > 0x7fffffff) return bsa::fail(c, "bad n");
  const double *in7[7] = {io->ptas, io->phdg, io->palt, io->pvs, io->bank, io->eps, io->accel};
  double *st6[6] = {io->tas, io->hdg, io->alt, io->vs, io->lat, io->lon};
  for (auto q : in7)
    if (!q) return bsa::fail(c, "bsa_kinematics: NULL input array");
  for (auto q : st6)
    if (!q) return bsa::fail(c, "bsa_kinematics: NULL state array");
  if (n == 0) return 0;
  BSA_HIP(c, hipSetDevice(c->device));
  const size_t N8 = (size_t)n * 8, NA = (N8 + 255) & ~size_t(255), NB = ((size_t)n + 255) & ~size_t(255);
  if (!bsa::ensure(c, c->kin_stage, NA * 23 + NB * 2, "kinematics staging")) return -1;
  char *b = (char *)c->kin_stage.p;
  double *din[7], *dst[6], *dout[10];
  for (int k = 0; k < 7; ++k) din[k] = (double *)(b + NA * k);
  for (int k = 0; k < 6; ++k) dst[k] = (double *)(b + NA * (7 + k));
  for (int k = 0; k < 10; ++k) dout[k] = (double *)(b + NA * (13 + k));
  uint8_t *dsw[2] = {(uint8_t *)(b + NA * 23), (uint8_t *)(b + NA * 23 + NB)};
  hipStream_t s = c->stream;
  for (int k = 0; k < 7; ++k) BSA_HIP(c, hipMemcpyAsync(din[k], in7[k], N8, hipMemcpyHostToDevice, s));
  for (int k = 0; k < 6; ++k) BSA_HIP(c, hipMemcpyAsync(dst[k], st6[k], N8, hipMemcpyHostToDevice, s));
  double *hout[10] = {io->ax, io->delspd, io->cas, io->mach, io->gsnorth, io->gseast, io->gs, io->trk,
                      io->coslat, io->az};
  uint8_t *hsw[2] = {io->swhdgsel, io->swaltsel};
  bsa::KinDev d;
  d.ptas = din[0]; d.phdg = din[1]; d.palt = din[2]; d.pvs = din[3];
  d.bank = din[4]; d.eps = din[5]; d.accel = din[6];
  d.tas = dst[0]; d.hdg = dst[1]; d.alt = dst[2]; d.vs = dst[3]; d.lat = dst[4]; d.lon = dst[5];
  d.ax = dout[0]; d.delspd = dout[1]; d.cas = dout[2]; d.mach = dout[3]; d.gsnorth = dout[4];
  d.gseast = dout[5]; d.gs = dout[6]; d.trk = dout[7]; d.coslat = dout[8]; d.az = dout[9];
  d.swhdgsel = dsw[0]; d.swaltsel = dsw[1];
  if (bsa::kin_device(c, n, simdt, winddim, windnorth, windeast, d)) return -1;
  for (int k = 0; k < 6; ++k) BSA_HIP(c, hipMemcpyAsync(st6[k], dst[k], N8, hipMemcpyDeviceToHost, s));
  for (int k = 0; k < 10; ++k)
    if (hout[k]) BSA_HIP(c, hipMemcpyAsync(hout[k], dout[k], N8, hipMemcpyDeviceToHost, s));
  for (int k = 0; k < 2; ++k)
    if (hsw[k]) BSA_HIP(c, hipMemcpyAsync(hsw[k], dsw[k], n, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipStreamSynchronize(s));
  return 0;
}
