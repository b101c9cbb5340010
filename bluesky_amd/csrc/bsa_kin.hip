// K4: fused kinematic integration of one sim step, one lane per aircraft
// (math in bsa_kin_math.h: traffic.py:425-483 + aero.py:62-147).
// HBM-bound: 13 fp64 reads + 16 fp64 + 2 byte writes per aircraft
// (234 B).
#include "bsa_kin_math.h"

#pragma clang fp contract(off)

namespace bsa {

__global__ __launch_bounds__(256) void k_kinematics(int n, double simdt, int winddim, double wn,
                                                    double we, WindField wf, KinDev d) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (winddim == 2) {  // traffic.py:463: getdata at the pre-step position
    kin::windfield_2d(wf, d.lat[k], d.lon[k], wn, we);
    winddim = 1;
  }
  kin::In s;
  s.tas = d.tas[k];
  s.hdg = d.hdg[k];
  s.alt = d.alt[k];
  s.vs = d.vs[k];
  s.lat = d.lat[k];
  s.lon = d.lon[k];
  s.ptas = d.ptas[k];
  s.phdg = d.phdg[k];
  s.palt = d.palt[k];
  s.pvs = d.pvs[k];
  s.bank = d.bank[k];
  s.eps = d.eps[k];
  s.accel = d.accel[k];
  const kin::Out o = kin::step(s, simdt, winddim, wn, we);
  d.tas[k] = o.tas;
  d.hdg[k] = o.hdg;
  d.alt[k] = o.alt;
  d.vs[k] = o.vs;
  d.lat[k] = o.lat;
  d.lon[k] = o.lon;
  if (d.ax) d.ax[k] = o.ax;
  if (d.delspd) d.delspd[k] = o.delspd;
  if (d.cas) d.cas[k] = o.cas;
  if (d.mach) d.mach[k] = o.mach;
  if (d.gsnorth) d.gsnorth[k] = o.gsnorth;
  if (d.gseast) d.gseast[k] = o.gseast;
  if (d.gs) d.gs[k] = o.gs;
  if (d.trk) d.trk[k] = o.trk;
  if (d.coslat) d.coslat[k] = o.coslat;
  if (d.az) d.az[k] = o.az;
  if (d.swhdgsel) d.swhdgsel[k] = o.swhdgsel;
  if (d.swaltsel) d.swaltsel[k] = o.swaltsel;
}

WindField wind_field(const Ctx *c) {
  WindField w;
  const double *p = (const double *)c->wfield.p;
  w.nvec = (int)c->wf_nvec;
  w.lat = p;
  w.lon = p ? p + c->wf_nvec : nullptr;
  w.vn = p ? p + 2 * c->wf_nvec : nullptr;
  w.ve = p ? p + 3 * c->wf_nvec : nullptr;
  return w;
}

int kin_device(Ctx *c, int64_t n, double simdt, int winddim, double vn, double ve, const KinDev &d) {
  if (n <= 0) return 0;
  if (winddim < 0 || winddim > 2) return fail(c, "winddim %d not supported (0, 1 or 2)", winddim);
  if (winddim == 2 && c->wf_nvec < 1) return fail(c, "winddim 2 needs a wind field (bsa_set_windfield)");
  hipLaunchKernelGGL(k_kinematics, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, (int)n,
                     simdt, winddim, vn, ve, wind_field(c), d);
  BSA_HIP(c, hipGetLastError());
  return 0;
}

}  // namespace bsa

extern "C" int bsa_set_windfield(bsa_ctx *cc, int64_t nvec, const double *lat, const double *lon,
                                 const double *vnorth, const double *veast) {
  bsa::Ctx *c = (bsa::Ctx *)cc;
  if (!c) return -1;
  if (nvec < 0 || nvec > (1 << 20)) return bsa::fail(c, "bad wind field size %lld", (long long)nvec);
  BSA_HIP(c, hipSetDevice(c->device));
  if (nvec == 0) {
    c->wf_nvec = 0;
    return 0;
  }
  if (!lat || !lon || !vnorth || !veast) return bsa::fail(c, "bsa_set_windfield: NULL array");
  if (!bsa::ensure(c, c->wfield, (size_t)nvec * 32, "wind field")) return -1;
  const double *src[4] = {lat, lon, vnorth, veast};
  for (int k = 0; k < 4; ++k)
    BSA_HIP(c, hipMemcpyAsync((double *)c->wfield.p + k * nvec, src[k], (size_t)nvec * 8, hipMemcpyHostToDevice,
                              c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  c->wf_nvec = nvec;
  return 0;
}

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
