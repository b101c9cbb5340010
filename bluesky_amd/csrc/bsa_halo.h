// Halo exchange pieces shared by bsa_halo.hip (plan, exchange) and bsa_cd.hip
// (the own-tile K0b fills the plan's zeroed buffers and box block; the halo
// K0b unpacks each received tile before preparing it) -- DESIGN.md 6.
#pragma once

#include "bsa_internal.h"

namespace bsa {

constexpr int kHaloMaxRanks = 16;
constexpr int kHaloMaxF = 8;  // fp64 arrays per halo row

struct HaloCaps {
  int scap[kHaloMaxRanks], rcap[kHaloMaxRanks];  // this rank's send / receive capacities [tiles]
  int hoff[kHaloMaxRanks];                       // flat halo list offset of each source
  unsigned long long soff[kHaloMaxRanks], roff[kHaloMaxRanks];  // region offsets in h_send / h_recv [B]
};

struct HaloFields {
  double *f[kHaloMaxF];  // lat lon trk gs alt vs gseast gsnorth (home order, full n)
  int nf;                // 6: gseast / gsnorth derived from gs / trk by the receiver
};

__host__ __device__ inline size_t halo_hdr_bytes(int cap) { return ((size_t)4 * (cap + 1) + 15) / 16 * 16; }
__host__ __device__ inline size_t halo_tile_bytes(int nf) { return (size_t)nf * kTile * 8; }

// What the own-tile K0b does for the plan (before the box all-gather): zero
// the plan's flag / demand / request words and write its tile boxes into the
// block sent to the other ranks (blk[tile - blk_base]; NULL in the probe).
struct HaloPre {
  unsigned *z[3];  // regions to zero (32-bit words)
  int zn[3];
  TileBox *blk;
  int blk_base;
};

// The halo K0b's unpack (exchange mode): workgroup j of the flat receive list
// first copies its tile's rows out of the received region (checked against
// this rank's own plan: a disagreement sets Counters::halo_miss and the tile
// is skipped, never prepared from stale rows).  rbuf == NULL: nothing to unpack.
struct HaloUnpack {
  const unsigned char *rbuf;
  HaloCaps cp;
  HaloFields fl;
  int R, n;
  const unsigned *count;  // the probe's dense list: its length (device; slots past it are unused), or NULL
};

// returns the tile to prepare (-1: none)
__device__ __forceinline__ int halo_unpack_tile(const HaloUnpack &u, int j, int want, Counters *cnt) {
  int q = 0;
  while (q + 1 < u.R && j >= u.cp.hoff[q + 1]) ++q;
  const int k = j - u.cp.hoff[q];
  const unsigned *hdr = reinterpret_cast<const unsigned *>(u.rbuf + u.cp.roff[q]);
  const int got = k < (int)hdr[0] ? (int)hdr[1 + k] : -1;
  if (got != want) {
    if (threadIdx.x == 0) cnt->halo_miss = 1;
    return -1;
  }
  if (got < 0) return -1;
  const int row = got * kTile + (int)threadIdx.x;
  if (row < u.n) {
    const double *src = reinterpret_cast<const double *>(u.rbuf + u.cp.roff[q] + halo_hdr_bytes(u.cp.rcap[q]) +
                                                         (size_t)k * halo_tile_bytes(u.fl.nf));
    for (int f = 0; f < u.fl.nf; ++f) u.fl.f[f][row] = src[f * kTile + threadIdx.x];
    if (u.fl.nf == 6) {  // K4' without wind: gseast / gsnorth = gs sin / cos(trk), bitwise the sender's
      const double gs = u.fl.f[3][row], trk = u.fl.f[2][row];
      double st, ct;
      sincos(trk * kD2R, &st, &ct);  // (as K4''s sincos of hdg)
      u.fl.f[7][row] = gs * ct;
      u.fl.f[6][row] = gs * st;
    }
  }
  return got;
}

// Tile-pair list reuse across the halo plan: the plan,
// its lists and K0d's list are rebuilt only when forced by the host or when
// some rank flags it -- a record of its own rows outside its drift budget
// (own K0b) or a resopairs request for a tile it does not hold (k_halo_req)
// -- the flags travelling with the box all-gather, so every rank takes the
// same decision (ctl[0]) from the same gathered words.  A rebuild plans on
// grown boxes.  tpr = 0: every detect plans (round-3 behaviour).
struct HaloTpr {
  int tpr, force;
  float dx, ds, dv;
  unsigned long long *ctl;  // tile-pair list control (Ctx::tpr_ctl): [0] the decision, read by K0d
  unsigned *myflag;         // this rank's flag word (in the box block; the probe: a control word)
};

// host side (bsa_halo.hip)
int halo_pre(Ctx *c, int64_t rb, int64_t re, HaloPre *hp, const HaloTpr *ht = nullptr);  // buffers; no launches
int halo_mid(Ctx *c, int64_t rb, int64_t re, HaloUnpack *hu, HaloTpr *ht = nullptr,
             bool hkeep = false, hipStream_t xs = nullptr);  // plan (+ exchange); hu->rbuf set in mode 1 (may
                                   // force ht); hkeep (HK kept plan): the exchange only -- no requests, box
                                   // all-gather or plan; xs (halo overlap): the send / recv on xs, after
                                   // the pack (on the context's stream; Ctx::ov_ev[0])
unsigned *halo_flag_word(Ctx *c);  // this rank's rebuild flag word (box block, or the probe's control word)

}  // namespace bsa
