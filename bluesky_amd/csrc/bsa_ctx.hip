// Context, device buffers, state upload and the C ABI entry points of
// include/bsaccel.h.  No exception crosses the ABI: every entry point
// returns a status and keeps its message in the context.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "bsa_internal.h"

namespace bsa {

static thread_local std::string g_create_error;

int fail(Ctx *c, const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf; else g_create_error = buf;
  return -1;
}

bool ensure(Ctx *c, DevBuf &b, size_t bytes, const char *what) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return true;
  if (b.p) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      fail(c, "sync before realloc of %s: %s", what, hipGetErrorString(e));
      return false;
    }
    (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
  }
  // round up to 2 MiB to limit reallocation churn
  size_t rounded = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
  hipError_t e = hipMalloc(&b.p, rounded);
  if (e != hipSuccess) {
    b.p = nullptr;
    fail(c, "hipMalloc(%zu) for %s failed: %s", rounded, what, hipGetErrorString(e));
    return false;
  }
  b.bytes = rounded;
  return true;
}

// ---------------------------------------------------------------- pinned host staging
// The drop-ins move 5-15 MB per call at 100k aircraft (bsa_sim_update's
// arrays, the pair lists, the ASAS outputs).  hipMemcpyAsync from pageable
// memory bounces through the runtime's own buffers one array at a time;
// here the host side is one parallel copy into a pinned buffer of the
// context and the device side ONE DMA of the whole batch.
namespace {
struct CopyPool {
  std::mutex use;  // one batch at a time (other callers copy on their own thread)
  std::mutex m;
  std::condition_variable cv, done_cv;
  std::vector<std::thread> th;
  std::vector<HostCopy> pieces;
  std::atomic<size_t> next{0}, done{0};
  unsigned gen = 0;
  int busy = 0;
  bool stop = false;
  CopyPool() {
    int nt = 8;
    if (const char *e = getenv("BSA_COPY_THREADS")) nt = atoi(e);
    const unsigned hw = std::thread::hardware_concurrency();
    nt = std::max(0, std::min(nt, (int)(hw > 1 ? hw - 1 : 0)));
    for (int k = 0; k < nt; ++k) th.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
  void work() {
    for (size_t k; (k = next.fetch_add(1)) < pieces.size();) {
      memcpy(pieces[k].dst, pieces[k].src, pieces[k].bytes);
      done.fetch_add(1);
    }
  }
  void loop() {
    unsigned seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m);
        cv.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        ++busy;
      }
      work();
      {
        std::lock_guard<std::mutex> lk(m);
        --busy;
      }
      done_cv.notify_all();
    }
  }
};
CopyPool &copy_pool() {
  static CopyPool *p = new CopyPool();  // (never destroyed: no join at static teardown)
  return *p;
}
}  // namespace

void host_copy(const HostCopy *jobs, int n) {
  constexpr size_t kPiece = size_t(256) << 10, kSmall = size_t(1) << 20;
  size_t total = 0;
  for (int k = 0; k < n; ++k) total += jobs[k].bytes;
  CopyPool &P = copy_pool();
  std::unique_lock<std::mutex> use(P.use, std::try_to_lock);
  if (total < kSmall || P.th.empty() || !use.owns_lock()) {
    for (int k = 0; k < n; ++k)
      if (jobs[k].bytes) memcpy(jobs[k].dst, jobs[k].src, jobs[k].bytes);
    return;
  }
  {
    // (under the lock, once no worker is inside work(): a late waker of the
    // last batch must never see the piece list change under it)
    std::unique_lock<std::mutex> lk(P.m);
    P.done_cv.wait(lk, [&] { return P.busy == 0; });
    P.pieces.clear();
    for (int k = 0; k < n; ++k)
      for (size_t o = 0; o < jobs[k].bytes; o += kPiece)
        P.pieces.push_back(HostCopy{(char *)jobs[k].dst + o, (const char *)jobs[k].src + o,
                                    std::min(kPiece, jobs[k].bytes - o)});
    P.next = 0;
    P.done = 0;
    ++P.gen;
  }
  P.cv.notify_all();
  P.work();
  std::unique_lock<std::mutex> lk(P.m);
  P.done_cv.wait(lk, [&] { return P.done.load() == P.pieces.size() && P.busy == 0; });
}

unsigned char *pin_stage(Ctx *c, size_t bytes) {
  if (c->pin_busy) {  // a DMA from the buffer may still run
    if (hipEventSynchronize(c->pin_ev) != hipSuccess) {
      fail(c, "pinned staging: event wait failed");
      return nullptr;
    }
    c->pin_busy = false;
  }
  if (c->pin_bytes < bytes) {
    if (c->pin) (void)hipHostFree(c->pin);
    c->pin = nullptr;
    c->pin_bytes = 0;
    const size_t rounded = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    if (hipHostMalloc(&c->pin, rounded, hipHostMallocDefault) != hipSuccess) {
      c->pin = nullptr;
      fail(c, "hipHostMalloc(%zu) for the pinned staging failed", rounded);
      return nullptr;
    }
    c->pin_bytes = rounded;
  }
  return (unsigned char *)c->pin;
}

int pin_issued(Ctx *c) {
  if (!c->pin_ev) BSA_HIP(c, hipEventCreateWithFlags(&c->pin_ev, hipEventDisableTiming));
  BSA_HIP(c, hipEventRecord(c->pin_ev, c->stream));
  c->pin_busy = true;
  return 0;
}

// Device-side gather of up to kGatherMax word arrays into one staging region
// (part k's wlen[k] words at word woff[k], 256-B aligned), so that a download
// is ONE DMA
__global__ __launch_bounds__(256) void k_gather_words(GatherParts g, unsigned *__restrict__ dst) {
  const unsigned long long nw = g.woff[g.n];
  for (unsigned long long w = blockIdx.x * 256ull + threadIdx.x; w < nw; w += (unsigned long long)gridDim.x * 256) {
    int p = 0;
    while (p + 1 < g.n && w >= g.woff[p + 1]) ++p;
    const unsigned long long i = w - g.woff[p];
    if (i < g.wlen[p]) dst[w] = g.src[p][i];
  }
}

// like ensure, but a grown buffer keeps its contents (persistent device state)
bool ensure_keep(Ctx *c, DevBuf &b, size_t bytes, const char *what) {
  if (bytes == 0) bytes = 16;
  if (b.bytes >= bytes) return true;
  DevBuf nb;
  if (!ensure(c, nb, bytes, what)) return false;
  if (b.p) {
    hipError_t e = hipMemcpyAsync(nb.p, b.p, b.bytes, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      fail(c, "copy on growth of %s: %s", what, hipGetErrorString(e));
      release(nb);
      return false;
    }
    release(b);
  }
  b = nb;
  return true;
}

void release(DevBuf &b) {
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
}

// the last detect's outputs as they lie on the device (rows of the detect, K2 order)
int download_pairs(Ctx *c, HostPairs &h) {
  const int64_t P = c->last_conf, L = c->last_los, R = c->last_re - c->last_rb;
  h.ci.resize((size_t)P);
  h.cj.resize((size_t)P);
  h.pay.resize((size_t)P * 5);
  h.li.resize((size_t)L);
  h.lj.resize((size_t)L);
  h.inconf.resize((size_t)R);
  h.tcpamax.resize((size_t)R);
  auto cp = [&](void *dst, const void *src, size_t bytes) -> int {
    if (bytes) BSA_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    return 0;
  };
  if (cp(h.ci.data(), c->out_ci.p, P * 4) || cp(h.cj.data(), c->out_cj.p, P * 4) ||
      cp(h.pay.data(), c->out_pay.p, P * 40) || cp(h.li.data(), c->out_li.p, L * 4) ||
      cp(h.lj.data(), c->out_lj.p, L * 4) || cp(h.inconf.data(), c->inconf.p, R) ||
      cp(h.tcpamax.data(), c->tcpamax.p, R * 8))
    return -1;
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

// Home rows -> aircraft indices: ci / li are home positions, cj / lj already
// indices, each row's pairs contiguous and ordered by cj (K2), so a stable
// sort of the pairs by their row's index gives np.where's row-major order
// (StateBasedCD.py:93-95); the per-row outputs of homes rb.. follow their
// rows' ascending indices.
// Linear in P + R (a comparison sort of the ~1.5e5 pairs took milliseconds):
// the rows' ascending-index order is known up front -- the sim's rows are
// [sim_rb, sim_re) with lpos_h, any other home slice is ordered once by a
// counting pass over its indices -- so each row's contiguous segment is moved
// to its row's place in that order.
void home_pairs_to_ids(const Ctx *c, int64_t rb, HostPairs &h) {
  const unsigned *H = c->h2id_h.data();
  const size_t P = h.ci.size(), L = h.li.size(), R = h.inconf.size();
  // byidx[k] = the home row (0..R-1, relative to rb) with the k-th smallest index
  std::vector<uint32_t> byidx(R);
  if (rb == c->sim_rb && (int64_t)R == c->sim_re - c->sim_rb && c->lpos_h.size() == R) {
    for (size_t r = 0; r < R; ++r) byidx[c->lpos_h[r]] = (uint32_t)r;
  } else {
    std::vector<std::pair<uint32_t, uint32_t>> ir(R);
    for (size_t r = 0; r < R; ++r) ir[r] = {H[rb + (int64_t)r], (uint32_t)r};
    std::sort(ir.begin(), ir.end());
    for (size_t k = 0; k < R; ++k) byidx[k] = ir[k].second;
  }
  // one list: segments by home row, then laid out in byidx order
  auto reorder = [&](std::vector<int32_t> &ri, size_t m, auto &&move) {
    std::vector<uint32_t> start(R + 1, 0u);
    for (size_t k = 0; k < m; ++k) start[(size_t)(ri[k] - rb) + 1]++;
    for (size_t r = 0; r < R; ++r) start[r + 1] += start[r];
    size_t at = 0;
    for (size_t k = 0; k < R; ++k) {
      const uint32_t r = byidx[k];
      for (uint32_t q = start[r]; q < start[r + 1]; ++q) move(at++, q);
    }
  };
  {
    std::vector<int32_t> ci(h.ci), cj(h.cj);
    std::vector<double> pay(h.pay);
    reorder(ci, P, [&](size_t to, uint32_t from) {
      h.ci[to] = (int32_t)H[ci[from]];
      h.cj[to] = cj[from];
      for (size_t f = 0; f < 5; ++f) h.pay[f * P + to] = pay[f * P + from];
    });
  }
  {
    std::vector<int32_t> li(h.li), lj(h.lj);
    reorder(li, L, [&](size_t to, uint32_t from) {
      h.li[to] = (int32_t)H[li[from]];
      h.lj[to] = lj[from];
    });
  }
  std::vector<uint8_t> inc(h.inconf);
  std::vector<double> tm(h.tcpamax);
  for (size_t k = 0; k < R; ++k) {
    h.inconf[k] = inc[byidx[k]];
    h.tcpamax[k] = tm[byidx[k]];
  }
}

// fetch_pairs of the resident sim's last CD call over this rank's rows: the
// lists are put into aircraft-index order on the device (rows in ascending
// index order, each row's contiguous segment moved whole), so the host copies
// them out once -- no host-side re-ordering pass over ~8 MB at 100k.
// k_fetch_lens: per row in index order its conflict / LoS segment lengths
// (then scanned into the new offsets) and its inconf / tcpamax.
__global__ __launch_bounds__(256) void k_fetch_lens(int R, const unsigned *__restrict__ byidx,
                                                    const unsigned *__restrict__ rowoff, unsigned *__restrict__ lens,
                                                    const uint8_t *__restrict__ inconf,
                                                    const unsigned long long *__restrict__ tcpamax,
                                                    uint8_t *__restrict__ o_inconf,
                                                    unsigned long long *__restrict__ o_tcpamax) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > R) return;
  if (k == R) {
    lens[R] = 0u;
    lens[2 * R + 1] = 0u;
    return;
  }
  const unsigned r = byidx[k];
  lens[k] = rowoff[r + 1] - rowoff[r];
  lens[R + 1 + k] = rowoff[R + 2 + r] - rowoff[R + 1 + r];
  o_inconf[k] = inconf[r];
  o_tcpamax[k] = tcpamax[r];
}
// one lane per row in index order: its segments to their new offsets, home
// rows mapped to aircraft indices
__global__ __launch_bounds__(256) void k_fetch_scatter(int R, int rb, const unsigned *__restrict__ byidx,
                                                       const unsigned *__restrict__ h2id,
                                                       const unsigned *__restrict__ rowoff,
                                                       const unsigned *__restrict__ noff, const int *__restrict__ cj,
                                                       const double *__restrict__ pay, const int *__restrict__ lj,
                                                       int *__restrict__ o_ci, int *__restrict__ o_cj,
                                                       double *__restrict__ o_pay, int *__restrict__ o_li,
                                                       int *__restrict__ o_lj) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= R) return;
  const unsigned r = byidx[k];
  const unsigned P = rowoff[R];
  const int id = (int)h2id[rb + (int)r];
  const unsigned s0 = rowoff[r], s1 = rowoff[r + 1], d0 = noff[k];
  for (unsigned s = s0; s < s1; ++s) {
    const unsigned d = d0 + (s - s0);
    o_ci[d] = id;
    o_cj[d] = cj[s];
#pragma unroll
    for (int f = 0; f < 5; ++f) o_pay[(size_t)f * P + d] = pay[(size_t)f * P + s];
  }
  const unsigned l0 = rowoff[R + 1 + r] - P, l1 = rowoff[R + 2 + r] - P, e0 = noff[R + 1 + k] - P;
  for (unsigned s = l0; s < l1; ++s) {
    o_li[e0 + (s - l0)] = id;
    o_lj[e0 + (s - l0)] = lj[s];
  }
}

static int fetch_home_device(Ctx *c, int32_t *ci, int32_t *cj, double *const dst5[5], int32_t *li, int32_t *lj,
                             uint8_t *inconf, double *tcpamax) {
  const int64_t P = c->last_conf, L = c->last_los, R = c->last_re - c->last_rb;
  auto al = [](size_t b) { return (b + 255) / 256 * 256; };
  const size_t o_ci = 0, o_cj = o_ci + al(P * 4), o_pay = o_cj + al(P * 4), o_li = o_pay + al(P * 40),
               o_lj = o_li + al(L * 4), o_inc = o_lj + al(L * 4), o_tm = o_inc + al(R), o_len = o_tm + al(R * 8),
               o_off = o_len + al(2 * (R + 1) * 4), total = o_off + al(2 * (R + 1) * 4);
  if (!ensure(c, c->fetch_stage, total, "fetch staging")) return -1;
  char *st = (char *)c->fetch_stage.p;
  const unsigned *rowoff = (const unsigned *)c->rowoff.p;
  hipLaunchKernelGGL(k_fetch_lens, dim3((unsigned)((R + 1 + 255) / 256)), dim3(256), 0, c->stream, (int)R,
                     (const unsigned *)c->lbyidx.p, rowoff, (unsigned *)(st + o_len), (const uint8_t *)c->inconf.p,
                     (const unsigned long long *)c->tcpamax.p, (uint8_t *)(st + o_inc),
                     (unsigned long long *)(st + o_tm));
  BSA_HIP(c, hipGetLastError());
  if (scan_excl(c, (const unsigned *)(st + o_len), (unsigned *)(st + o_off), (int)(2 * (R + 1)))) return -1;
  hipLaunchKernelGGL(k_fetch_scatter, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, c->stream, (int)R,
                     (int)c->last_rb, (const unsigned *)c->lbyidx.p, (const unsigned *)c->h2id.p, rowoff,
                     (const unsigned *)(st + o_off), (const int *)c->out_cj.p, (const double *)c->out_pay.p,
                     (const int *)c->out_lj.p, (int *)(st + o_ci), (int *)(st + o_cj), (double *)(st + o_pay),
                     (int *)(st + o_li), (int *)(st + o_lj));
  BSA_HIP(c, hipGetLastError());
  // the re-ordered lists [0, o_len) in ONE DMA into the pinned staging, then
  // one parallel host copy into the caller's arrays
  unsigned char *pin = pin_stage(c, o_len);
  if (!pin) return -1;
  BSA_HIP(c, hipMemcpyAsync(pin, st, o_len, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  HostCopy jobs[11];
  int nj = 0;
  auto cp = [&](void *dst, size_t off, size_t bytes) {
    if (dst && bytes) jobs[nj++] = HostCopy{dst, pin + off, bytes};
  };
  cp(ci, o_ci, P * 4);
  cp(cj, o_cj, P * 4);
  cp(li, o_li, L * 4);
  cp(lj, o_lj, L * 4);
  cp(inconf, o_inc, R);
  cp(tcpamax, o_tm, R * 8);
  for (int f = 0; f < 5; ++f) cp(dst5[f], o_pay + (size_t)f * P * 8, P * 8);
  host_copy(jobs, nj);
  return 0;
}

static int upload6(Ctx *c, DevBuf *dst, int64_t n, const double *const src[6]) {
  static const char *names[6] = {"lat", "lon", "trk", "gs", "alt", "vs"};
  for (int k = 0; k < 6; ++k) {
    if (!src[k]) return fail(c, "NULL %s array", names[k]);
    if (!ensure(c, dst[k], (size_t)n * 8, names[k])) return -1;
  }
  if (!n) return 0;
  // one parallel host copy into the pinned staging, then the six DMAs
  const size_t nb = (size_t)n * 8;
  unsigned char *pin = pin_stage(c, 6 * nb);
  if (!pin) return -1;
  HostCopy jobs[6];
  for (int k = 0; k < 6; ++k) jobs[k] = HostCopy{pin + k * nb, src[k], nb};
  host_copy(jobs, 6);
  for (int k = 0; k < 6; ++k)
    BSA_HIP(c, hipMemcpyAsync(dst[k].p, pin + k * nb, nb, hipMemcpyHostToDevice, c->stream));
  return pin_issued(c);
}

}  // namespace bsa

using bsa::Ctx;

struct bsa_ctx : Ctx {};

extern "C" {

int bsa_abi_version(void) { return BSA_ABI_VERSION; }

int bsa_device_count(void) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e == hipErrorNoDevice) return 0;
  if (e != hipSuccess) return -1;
  return n;
}

bsa_ctx *bsa_create(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    bsa::fail(nullptr, "no HIP device available (%s)", hipGetErrorString(e));
    return nullptr;
  }
  if (device < 0 || device >= n) {
    bsa::fail(nullptr, "device %d out of range [0, %d)", device, n);
    return nullptr;
  }
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    bsa::fail(nullptr, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
    return nullptr;
  }
  bsa_ctx *c = new (std::nothrow) bsa_ctx();
  if (!c) {
    bsa::fail(nullptr, "out of host memory");
    return nullptr;
  }
  c->device = device;
  // longest prefilter items first (bsa_cd.hip HeavyArgs): the listing
  // threshold, or off (BSA_PF_HEAVY=0); results never depend on it
  if (const char *v = getenv("BSA_PF_HEAVY_US")) {
    c->hv_us = atof(v);
    c->hv_us_env = true;
  }
  if (getenv("BSA_PF_HEAVY") && atoi(getenv("BSA_PF_HEAVY")) == 0) c->hv_us = -1.0;
  if (const char *v = getenv("BSA_PF_HEAVY_X")) c->hv_x = atof(v);
  // host-known tile-pair list decisions (Ctx::hk_*; BSA_HK=0 off, BSA_HK_F the
  // prediction fraction); results never depend on them
  if (getenv("BSA_HK") && atoi(getenv("BSA_HK")) == 0) c->hk_on = false;
  if (const char *v = getenv("BSA_HK_F")) {
    const float f = (float)atof(v);
    if (f > 0.f && f <= 1.f) c->hk_f = f;
  }
  // halo overlap (Ctx::ov_mode): 0 off (default), 1 exchange mode, 2 also the probe
  if (const char *v = getenv("BSA_HALO_OVERLAP")) c->ov_mode = std::min(std::max(atoi(v), 0), 2);
  if (const char *v = getenv("BSA_OV_EVFLAGS")) c->ov_evflags = (unsigned)atoi(v);
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    bsa::fail(nullptr, "hipStreamCreate: %s", hipGetErrorString(e));
    delete c;
    return nullptr;
  }
  return c;
}

void bsa_destroy(bsa_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  if (c->pin) (void)hipHostFree(c->pin);
  if (c->pin_ev) (void)hipEventDestroy(c->pin_ev);
  if (c->hk_host) (void)hipHostFree(c->hk_host);
  c->hk_host = c->hk_hdev = nullptr;
  c->pin = nullptr;
  c->pin_ev = nullptr;
  bsa::DevBuf *all[] = {&c->rowrec, &c->colrec, &c->pfrow, &c->pfcol, &c->counters, &c->cand,
                        &c->ckey, &c->cval, &c->ckey2, &c->cval2, &c->cpay, &c->kbuck, &c->lkey, &c->lkey2,
                        &c->out_ci, &c->out_cj, &c->out_li, &c->out_lj, &c->out_pay, &c->inconf,
                        &c->tcpamax, &c->sort_tmp, &c->seg, &c->mvp_stage, &c->kin_stage, &c->mvp_pdv, &c->mvp_pfl, &c->mvp_rowdv,
                        &c->pfvrow, &c->pfvcol, &c->pfprow, &c->pfpcol, &c->key_r, &c->idx_r, &c->key_r2, &c->perm_r,
                        &c->key_c, &c->idx_c, &c->key_c2, &c->perm_c, &c->tbox_r, &c->tbox_c,
                        &c->gbox_r, &c->gbox_c, &c->sbox_c, &c->workq, &c->workq2, &c->counters2, &c->rowcnt, &c->rowoff,
                        &c->cflag, &c->stats,
                        &c->tilepairs, &c->scan_ws, &c->snap_build, &c->snap_cur, &c->reuse_ctl, &c->reuse_use,
                        &c->geo_in, &c->geo_pts, &c->geo_out, &c->wfield,
                        &c->hv_cost, &c->hv_flag, &c->hv_list[0], &c->hv_list[1], &c->hv_list[2], &c->hv_list[3],
                        &c->hv_cnt, &c->nonfin, &c->rownf};
  for (auto *b : all) bsa::release(*b);
  bsa::sim_release(c);
  bsa::feed_release(c);
  for (int k = 0; k < 6; ++k) {
    bsa::release(c->own[k]);
    bsa::release(c->intr[k]);
  }
  for (hipEvent_t e : c->evpool)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->geo_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ov_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->xstream) {
    (void)hipStreamSynchronize(c->xstream);
    (void)hipStreamDestroy(c->xstream);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char *bsa_last_error(const bsa_ctx *c) {
  return c ? c->err.c_str() : bsa::g_create_error.c_str();
}

int bsa_sync(bsa_ctx *c) {
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

int bsa_set_state(bsa_ctx *c, int64_t n, const double *lat, const double *lon, const double *trk,
                  const double *gs, const double *alt, const double *vs) {
  if (!c) return -1;
  if (n < 0) return bsa::fail(c, "negative n");
  BSA_HIP(c, hipSetDevice(c->device));
  c->sim_ready = false;  // a new state replaces any resident sim
  c->sim_prepped = false;
  c->tpr_valid = false;  // (tile-pair list / halo plan reuse: rebuilt at the next detect)
  c->home = false;       // ... and its home order: aircraft-index order again
  const double *src[6] = {lat, lon, trk, gs, alt, vs};
  if (n == 0) {
    c->n = 0;
    c->has_intruder = false;
    c->have_pairs = false;
    return 0;
  }
  if (bsa::upload6(c, c->own, n, src)) return -1;
  c->n = n;
  c->has_intruder = false;
  c->have_pairs = false;
  return 0;
}

int bsa_set_intruder(bsa_ctx *c, int64_t n, const double *lat, const double *lon, const double *trk,
                     const double *gs, const double *alt, const double *vs) {
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  if (n == 0) {
    c->has_intruder = false;
    return 0;
  }
  if (n != c->n) return bsa::fail(c, "intruder n=%lld != ownship n=%lld", (long long)n, (long long)c->n);
  const double *src[6] = {lat, lon, trk, gs, alt, vs};
  if (bsa::upload6(c, c->intr, n, src)) return -1;
  c->has_intruder = true;
  c->have_pairs = false;
  return 0;
}

int bsa_detect(bsa_ctx *c, double rpz, double hpz, double tla, int flags, int64_t row_begin,
               int64_t row_end, int64_t *n_conf, int64_t *n_los) {
  if (!c) return -1;
  if (!n_conf || !n_los) return bsa::fail(c, "NULL count pointer");
  if (c->home)
    return bsa::fail(c, "bsa_detect on a context whose state is a resident sim's (home order): "
                        "bsa_set_state first, or use another context");
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::detect(c, rpz, hpz, tla, flags, row_begin, row_end, n_conf, n_los);
}

int bsa_fetch_pairs(bsa_ctx *c, int32_t *ci, int32_t *cj, double *qdr, double *dist, double *tcpa,
                    double *tinconf, double *dcpa, int32_t *li, int32_t *lj, uint8_t *inconf,
                    double *tcpamax) {
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  if (bsa::sim_adopt_pairs(c)) return -1;
  if (!c->have_pairs) return bsa::fail(c, "no detect results to fetch");
  const int64_t P = c->last_conf, L = c->last_los, R = c->last_re - c->last_rb;
  const double *pay = (const double *)c->out_pay.p;
  if (dcpa && !(c->last_flags & BSA_FLAG_WITH_DCPA)) return bsa::fail(c, "dcpa requested without BSA_FLAG_WITH_DCPA");
  if (c->last_home && c->last_rb == c->sim_rb && c->last_re == c->sim_re && c->lbyidx.p &&
      c->last_re > c->last_rb) {  // the sim's own rows: re-ordered on the device
    double *dst5[5] = {qdr, dist, tcpa, tinconf, dcpa};
    return bsa::fetch_home_device(c, ci, cj, dst5, li, lj, inconf, tcpamax);
  }
  if (c->last_home) {  // another home slice (bsa_sim_detect_rows): translated on the host
    bsa::HostPairs h;
    if (bsa::download_pairs(c, h)) return -1;
    bsa::home_pairs_to_ids(c, c->last_rb, h);
    auto put = [](void *dst, const void *src, size_t bytes) {
      if (dst && bytes) memcpy(dst, src, bytes);
    };
    put(ci, h.ci.data(), P * 4);
    put(cj, h.cj.data(), P * 4);
    double *dst5[5] = {qdr, dist, tcpa, tinconf, dcpa};
    for (int f = 0; f < 5; ++f) put(dst5[f], h.pay.data() + (size_t)f * P, P * 8);
    put(li, h.li.data(), L * 4);
    put(lj, h.lj.data(), L * 4);
    put(inconf, h.inconf.data(), R);
    put(tcpamax, h.tcpamax.data(), R * 8);
    return 0;
  }
  // every requested array by DMA into the pinned staging, then one parallel
  // host copy into the caller's arrays
  struct {
    void *dst;
    const void *src;
    size_t bytes;
  } part[11] = {{ci, c->out_ci.p, (size_t)P * 4},  {cj, c->out_cj.p, (size_t)P * 4},   {qdr, pay, (size_t)P * 8},
                {dist, pay + P, (size_t)P * 8},     {tcpa, pay + 2 * P, (size_t)P * 8}, {tinconf, pay + 3 * P, (size_t)P * 8},
                {dcpa, pay + 4 * P, (size_t)P * 8}, {li, c->out_li.p, (size_t)L * 4},  {lj, c->out_lj.p, (size_t)L * 4},
                {inconf, c->inconf.p, (size_t)R},   {tcpamax, c->tcpamax.p, (size_t)R * 8}};
  // gathered on the device into one staging region (one launch), ONE DMA
  // into the pinned staging, one parallel host copy into the caller's arrays
  bsa::GatherParts g{};
  bsa::HostCopy jobs[11];
  size_t off = 0;
  for (auto &q : part) {
    if (!q.dst || !q.bytes) continue;
    g.src[g.n] = (const unsigned *)q.src;
    g.woff[g.n] = off / 4;
    g.wlen[g.n] = (q.bytes + 3) / 4;  // (a byte array's last word: inside its 2 MiB-rounded allocation)
    jobs[g.n] = bsa::HostCopy{q.dst, nullptr, q.bytes};
    g.n++;
    off += (q.bytes + 255) / 256 * 256;
  }
  g.woff[g.n] = off / 4;
  if (!g.n) return 0;
  if (!bsa::ensure(c, c->fetch_stage, off, "fetch staging")) return -1;
  unsigned char *pin = bsa::pin_stage(c, off);
  if (!pin) return -1;
  hipLaunchKernelGGL(bsa::k_gather_words, dim3((unsigned)std::min<size_t>((off / 4 + 255) / 256, 2048)), dim3(256), 0,
                     c->stream, g, (unsigned *)c->fetch_stage.p);
  BSA_HIP(c, hipGetLastError());
  BSA_HIP(c, hipMemcpyAsync(pin, c->fetch_stage.p, off, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < g.n; ++k) jobs[k].src = pin + g.woff[k] * 4;
  bsa::host_copy(jobs, g.n);
  return 0;
}

int bsa_last_candidates(bsa_ctx *c, int64_t *n_candidates) {
  if (!c || !n_candidates) return -1;
  *n_candidates = c->last_cand;
  return 0;
}

int bsa_set_candidate_capacity(bsa_ctx *c, int64_t capacity) {
  if (!c) return -1;
  if (capacity < 1) return bsa::fail(c, "candidate capacity must be >= 1");
  const unsigned long long s = bsa::kCandShards;
  c->cand_cap = ((unsigned long long)capacity + s - 1) / s * s;
  if (c->bk_cap) c->bk_cap = (unsigned long long)capacity;  // resident-sim resopairs (grows the same way)
  return 0;
}

int bsa_set_row_bucket(bsa_ctx *c, int width) {
  if (!c) return -1;
  if (width < 0 || width > 64) return bsa::fail(c, "row bucket width must be in [0, 64]");
  c->k2_bucket = width;
  return 0;
}

int bsa_set_exact_fusion(bsa_ctx *c, int on, int max_records) {
  if (!c) return -1;
  if (max_records < 0 || max_records > bsa::kFuseRecsMax)
    return bsa::fail(c, "max_records must be in [0, %d]", bsa::kFuseRecsMax);
  c->fuse_on = on != 0;
  c->fuse_recs = max_records;
  return 0;
}

int bsa_exact_fusion_stats(bsa_ctx *c, int64_t *out3) {
  if (!c || !out3) return -1;
  out3[0] = c->fuse_count;
  out3[1] = c->fuse_retries;
  out3[2] = c->last_fused ? 1 : 0;
  return 0;
}

int bsa_set_candidate_reuse(bsa_ctx *c, int on, double sigma_h, double sigma_v) {
  if (!c) return -1;
  if (on && !(sigma_h > 0.0 && sigma_h < 1e6 && sigma_v > 0.0 && sigma_v < 1e5))
    return bsa::fail(c, "reuse budgets must be positive (sigma_h < 1000 km, sigma_v < 100 km)");
  c->reuse_on = on != 0;
  if (on) {
    c->reuse_sh = sigma_h;
    c->reuse_sv = sigma_v;
  }
  c->reuse_valid = false;  // the next detect builds
  return 0;
}

int bsa_sim_comm_stats(bsa_ctx *c, int64_t *out3) {
  if (!c || !out3) return -1;
  out3[0] = c->comm_calls;
  out3[1] = c->comm_tx;
  out3[2] = c->comm_rx;
  return 0;
}

int bsa_set_tile_reuse(bsa_ctx *c, int on, double sigma_h, double sigma_v) {
  if (!c) return -1;
  if (on && !(sigma_h > 0.0 && sigma_h < 1e5 && sigma_v > 0.0 && sigma_v < 1e4))
    return bsa::fail(c, "tile reuse budgets must be positive (sigma_h < 100 km, sigma_v < 10 km)");
  c->tpr_on = on != 0;
  if (on) {
    c->tpr_dx = (float)(sigma_h / 6.3e6);       // chord units (a unit-vector axis moves <= its chord)
    c->tpr_ds = (float)(sigma_h / 6.3e6 / 20);  // reach: |V| T/2 changes with the speed, slowly
    c->tpr_dv = (float)sigma_v;
  }
  c->tpr_valid = false;  // the next detect builds
  return 0;
}

int bsa_tile_reuse_stats(bsa_ctx *c, int64_t *out2) {
  if (!c || !out2) return -1;
  unsigned long long w[8] = {0};
  if (c->tpr_ctl.p) {
    BSA_HIP(c, hipSetDevice(c->device));
    BSA_HIP(c, hipMemcpyAsync(w, c->tpr_ctl.p, sizeof(w), hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
  }
  out2[0] = (int64_t)w[3];
  out2[1] = (int64_t)w[4];
  return 0;
}

int bsa_set_hk(bsa_ctx *c, int on, double f) {
  if (!c) return -1;
  if (!(f > 0.0 && f <= 4.0)) return bsa::fail(c, "HK prediction fraction must be in (0, 4]");
  c->hk_on = on != 0;
  c->hk_f = (float)f;
  c->hk_ok = false;  // (the next host-decided detect builds)
  return 0;
}

int bsa_set_halo_overlap(bsa_ctx *c, int mode) {
  if (!c) return -1;
  if (mode < 0 || mode > 2) return bsa::fail(c, "halo overlap mode must be 0, 1 or 2");
  c->ov_mode = mode;
  return 0;
}

int bsa_halo_overlap_count(bsa_ctx *c, int64_t *out1) {
  if (!c || !out1) return -1;
  out1[0] = c->ov_count;
  return 0;
}

int bsa_hk_stats(bsa_ctx *c, int64_t *out6) {
  if (!c || !out6) return -1;
  out6[0] = c->hk_keeps;
  out6[1] = c->hk_builds;
  out6[2] = c->hk_waits;
  out6[3] = c->hk_stale;
  out6[4] = c->hk_cool;
  out6[5] = c->hk_on ? 1 : 0;
  return 0;
}

int bsa_reuse_stats(bsa_ctx *c, int64_t *builds, int64_t *detects) {
  if (!c || !builds || !detects) return -1;
  unsigned long long st[8] = {0};
  if (c->stats.p) {
    BSA_HIP(c, hipSetDevice(c->device));
    BSA_HIP(c, hipMemcpyAsync(st, c->stats.p, sizeof(st), hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
  }
  *builds = (int64_t)st[4];
  *detects = (int64_t)st[3];
  return 0;
}

int bsa_reuse_budget_use(bsa_ctx *c, double *use2) {
  if (!c || !use2) return -1;
  use2[0] = use2[1] = 0.0;
  if (!c->reuse_use.p || c->reuse_n <= 0) return 0;
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<float> u((size_t)((c->reuse_n + 63) / 64) * 2);
  BSA_HIP(c, hipMemcpyAsync(u.data(), c->reuse_use.p, u.size() * 4, hipMemcpyDeviceToHost, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  for (size_t k = 0; k < u.size(); k += 2) {
    use2[0] = std::max(use2[0], (double)u[k]);
    use2[1] = std::max(use2[1], (double)u[k + 1]);
  }
  return 0;
}

int bsa_last_tiles(bsa_ctx *c, int64_t *kept, int64_t *total, int64_t *groups) {
  if (!c || !kept || !total || !groups) return -1;
  *kept = c->last_tiles;
  *total = c->last_tiles_total;
  *groups = c->last_groups;
  return 0;
}

// stage durations [ms] of one recorded detect: K0 (zero, order, records,
// boxes, tile pairs), K1a prefilter, K1b exact, K2 (scan, scatter, rank), total
static int event_set_ms(bsa::Ctx *c, int set, double *ms5) {
  hipEvent_t *ev = &c->evpool[5 * (size_t)set];
  BSA_HIP(c, hipEventSynchronize(ev[4]));
  float t;
  for (int k = 0; k < 4; ++k) {
    BSA_HIP(c, hipEventElapsedTime(&t, ev[k], ev[k + 1]));
    ms5[k] = t;
  }
  BSA_HIP(c, hipEventElapsedTime(&t, ev[0], ev[4]));
  ms5[4] = t;
  return 0;
}

int bsa_last_timings(bsa_ctx *c, double *ms5) {
  if (!c || !ms5) return -1;
  if (!c->ev_valid) return bsa::fail(c, "no timed detect yet");
  BSA_HIP(c, hipSetDevice(c->device));
  return event_set_ms(c, c->ev_last, ms5);
}

int bsa_timing_reset(bsa_ctx *c) {
  if (!c) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  c->ev_sets = 0;
  c->ev_count = 0;
  c->ev_valid = false;
  c->comm_calls = c->comm_tx = c->comm_rx = 0;
  if (!bsa::ensure(c, c->stats, 8 * 8, "detect statistics")) return -1;
  BSA_HIP(c, hipMemsetAsync(c->stats.p, 0, 8 * 8, c->stream));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  return 0;
}

int bsa_set_timing_sample(bsa_ctx *c, int every) {
  if (!c) return -1;
  if (every < 0) return bsa::fail(c, "timing sample interval must be >= 0");
  c->ev_every = every;
  c->ev_count = 0;
  return 0;
}

int bsa_timing_summary(bsa_ctx *c, double *ms5, int64_t *stats4) {
  if (!c || !ms5 || !stats4) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < 5; ++k) ms5[k] = 0.0;
  const int sets = std::min(c->ev_sets, bsa::kEvSets);
  for (int q = 0; q < sets; ++q) {
    double m[5];
    if (event_set_ms(c, q, m)) return -1;
    for (int k = 0; k < 5; ++k) ms5[k] += m[k] / sets;
  }
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c->stats.p) BSA_HIP(c, hipMemcpy(st, c->stats.p, sizeof(st), hipMemcpyDeviceToHost));
  for (int k = 0; k < 4; ++k) stats4[k] = (int64_t)st[k];
  return 0;
}

}  // extern "C"
