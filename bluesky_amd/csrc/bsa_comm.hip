// Collectives of the row-sharded resident sim, behind one
// interface with two transports:
//
//  * RCCL (ncclComm_t over xGMI): one process per GPU -- the production path
//    (bsa_comm_init with an id from bsa_comm_unique_id).
//  * an in-process group (bsa_group_*): several contexts in ONE process, each
//    driven by its own host thread, exchanging through device-to-device copies
//    ordered by HIP events and a host barrier.  RCCL rejects two ranks on one
//    GPU, so this is how the nranks > 1 code paths (k_pack / k_unpack, the gate
//    all-reduce, the rank-order pair gather, the global unique-pair counts) run
//    and are checked on a one-GPU box; it also serves a single process that
//    drives several GPUs from several threads.
//
// Every collective is stream-ordered like RCCL's: it is enqueued on the
// context's stream behind the work that produces its input, and later work on
// that stream sees its output; only the host-value reductions synchronise.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>

#include "bsa_internal.h"

namespace bsa {

#define BSA_NCCL(c, call)                                                                     \
  do {                                                                                        \
    ncclResult_t r_ = (call);                                                                 \
    if (r_ != ncclSuccess)                                                                    \
      return ::bsa::fail((c), "%s failed: %s (%s:%d)", #call, ncclGetErrorString(r_), __FILE__, \
                         __LINE__);                                                           \
  } while (0)

constexpr int kMaxGroup = 16;

struct Group {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long long phase = 0;
  bool broken = false;
  bool destroy_pending = false;           // bsa_group_destroy while members were still joined
  Ctx *ctx[kMaxGroup] = {};
  DevBuf slot[kMaxGroup];                 // each rank's published copy (its own device)
  hipEvent_t pub[kMaxGroup] = {}, done[kMaxGroup] = {};
  std::vector<double> host[kMaxGroup];    // host-value exchange
  std::vector<size_t> hlen[kMaxGroup];    // comm_halo: each rank's send lengths and offsets (2 R)
};

// host barrier of the group; false (and the group marked broken) after 120 s
// or when another rank gave up, so an error on one rank cannot hang the others
static bool barrier(Ctx *c) {
  Group *g = c->group;
  std::unique_lock<std::mutex> lk(g->m);
  if (g->broken) return fail(c, "in-process group broken by another rank"), false;
  const unsigned long long ph = g->phase;
  if (++g->arrived == g->n) {
    g->arrived = 0;
    g->phase++;
    g->cv.notify_all();
    return true;
  }
  const bool ok = g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->phase != ph || g->broken; });
  if (!ok || g->broken) {
    g->broken = true;
    g->cv.notify_all();
    fail(c, "in-process group barrier timed out or broken (rank %d)", c->rank);
    return false;
  }
  return true;
}

// the members' `done` events as they are now (under the lock: a rank that
// has not joined yet -- its thread still before bsa_comm_init_group -- has
// none, and has read no slot either, so there is nothing to wait for)
static void done_events(Group *g, hipEvent_t *ev) {
  std::lock_guard<std::mutex> lk(g->m);
  for (int q = 0; q < g->n; ++q) ev[q] = g->done[q];
}

// rank r publishes `bytes` from device `src` into its slot (after every rank
// finished reading the previous collective's slots), then waits for all slots
static int publish(Ctx *c, const void *src, size_t bytes) {
  Group *g = c->group;
  const int r = c->rank;
  hipEvent_t done[kMaxGroup];
  done_events(g, done);
  for (int q = 0; q < g->n; ++q)
    if (done[q]) BSA_HIP(c, hipStreamWaitEvent(c->stream, done[q], 0));
  if (g->slot[r].bytes < bytes) {
    for (int q = 0; q < g->n; ++q)
      if (done[q]) BSA_HIP(c, hipEventSynchronize(done[q]));
    if (!ensure(c, g->slot[r], bytes, "group slot")) return -1;
  }
  if (bytes) BSA_HIP(c, hipMemcpyAsync(g->slot[r].p, src, bytes, hipMemcpyDeviceToDevice, c->stream));
  BSA_HIP(c, hipEventRecord(g->pub[r], c->stream));
  if (!barrier(c)) return -1;
  for (int q = 0; q < g->n; ++q) BSA_HIP(c, hipStreamWaitEvent(c->stream, g->pub[q], 0));
  return 0;
}

static int retire(Ctx *c) {
  Group *g = c->group;
  BSA_HIP(c, hipEventRecord(g->done[c->rank], c->stream));
  return barrier(c) ? 0 : -1;
}

struct SlotPtrs {
  const unsigned long long *p[kMaxGroup];
};
__global__ void k_max_u64_slots(unsigned long long *out, int count, int nq, SlotPtrs s) {
  const int k = threadIdx.x;
  if (k >= count) return;
  unsigned long long v = 0;
  for (int q = 0; q < nq; ++q) v = s.p[q][k] > v ? s.p[q][k] : v;
  out[k] = v;
}

bool comm_multi(const Ctx *c) { return c->nranks > 1 && (c->comm || c->group); }

static void account(Ctx *c, size_t tx, size_t rx) {
  c->comm_calls++;
  c->comm_tx += (int64_t)tx;
  c->comm_rx += (int64_t)rx;
}

int comm_allgather(Ctx *c, const void *send, void *recv, size_t bytes) {
  if (!comm_multi(c)) {
    if (bytes && recv != send) BSA_HIP(c, hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, c->stream));
    return 0;
  }
  account(c, bytes, bytes * (size_t)(c->nranks - 1));
  if (c->comm) {
    BSA_NCCL(c, ncclAllGather(send, recv, bytes, ncclUint8, (ncclComm_t)c->comm, c->stream));
    return 0;
  }
  Group *g = c->group;
  if (publish(c, send, bytes)) return -1;
  for (int q = 0; q < g->n; ++q)
    if (bytes)
      BSA_HIP(c, hipMemcpyAsync((char *)recv + (size_t)q * bytes, g->slot[q].p, bytes, hipMemcpyDeviceToDevice,
                                c->stream));
  return retire(c);
}

// In-place all-gather of nf fp64 arrays, each at least nranks * rpr long:
// rank q's block [q rpr, (q + 1) rpr) of every array reaches every rank (the
// resident sim's home ranges are contiguous, so nothing is packed or
// unpacked).  RCCL: nf in-place ncclAllGather fused in one group.
int comm_allgather_inplace(Ctx *c, double *const *f, int nf, size_t rpr) {
  if (!comm_multi(c) || rpr == 0 || nf <= 0) return 0;
  account(c, rpr * 8 * nf, rpr * 8 * nf * (size_t)(c->nranks - 1));
  if (c->comm) {
    BSA_NCCL(c, ncclGroupStart());
    for (int k = 0; k < nf; ++k)
      BSA_NCCL(c, ncclAllGather(f[k] + (size_t)c->rank * rpr, f[k], rpr, ncclDouble, (ncclComm_t)c->comm, c->stream));
    BSA_NCCL(c, ncclGroupEnd());
    return 0;
  }
  // in-process group: this rank's blocks into its slot, then every peer's
  // blocks out of theirs
  Group *g = c->group;
  const size_t blk = rpr * 8;
  if (!ensure(c, c->g_send, blk * nf, "gather send")) return -1;
  for (int k = 0; k < nf; ++k)
    BSA_HIP(c, hipMemcpyAsync((char *)c->g_send.p + k * blk, f[k] + (size_t)c->rank * rpr, blk,
                              hipMemcpyDeviceToDevice, c->stream));
  if (publish(c, c->g_send.p, blk * nf)) return -1;
  for (int q = 0; q < g->n; ++q) {
    if (q == c->rank) continue;
    for (int k = 0; k < nf; ++k)
      BSA_HIP(c, hipMemcpyAsync(f[k] + (size_t)q * rpr, (const char *)g->slot[q].p + k * blk, blk,
                                hipMemcpyDeviceToDevice, c->stream));
  }
  return retire(c);
}

int comm_allreduce_max_u64(Ctx *c, unsigned long long *buf, int count) {
  if (!comm_multi(c) || count <= 0) return 0;
  if (count > 256) return fail(c, "device max all-reduce of %d words", count);
  account(c, (size_t)count * 8, (size_t)count * 8);
  if (c->comm) {
    BSA_NCCL(c, ncclAllReduce(buf, buf, (size_t)count, ncclUint64, ncclMax, (ncclComm_t)c->comm, c->stream));
    return 0;
  }
  Group *g = c->group;
  if (publish(c, buf, (size_t)count * 8)) return -1;
  // stage every peer's slot into this rank's scratch with copies (the group
  // may span devices without peer access), then reduce locally
  const size_t b = (size_t)count * 8;
  if (!ensure(c, c->red, b * g->n, "reduction scratch")) return -1;
  SlotPtrs s{};
  for (int q = 0; q < g->n; ++q) {
    BSA_HIP(c, hipMemcpyAsync((char *)c->red.p + q * b, g->slot[q].p, b, hipMemcpyDeviceToDevice, c->stream));
    s.p[q] = (const unsigned long long *)((const char *)c->red.p + q * b);
  }
  hipLaunchKernelGGL(k_max_u64_slots, dim3(1), dim3(256), 0, c->stream, buf, count, g->n, s);
  BSA_HIP(c, hipGetLastError());
  return retire(c);
}

int comm_allreduce_host(Ctx *c, double *v, int count, bool max) {
  if (!comm_multi(c) || count <= 0) return 0;
  if (c->comm) {
    if (!ensure(c, c->red, (size_t)count * 8, "reduction scratch")) return -1;
    BSA_HIP(c, hipMemcpyAsync(c->red.p, v, (size_t)count * 8, hipMemcpyHostToDevice, c->stream));
    BSA_NCCL(c, ncclAllReduce(c->red.p, c->red.p, (size_t)count, ncclDouble, max ? ncclMax : ncclSum,
                              (ncclComm_t)c->comm, c->stream));
    BSA_HIP(c, hipMemcpyAsync(v, c->red.p, (size_t)count * 8, hipMemcpyDeviceToHost, c->stream));
    BSA_HIP(c, hipStreamSynchronize(c->stream));
    return 0;
  }
  Group *g = c->group;
  BSA_HIP(c, hipStreamSynchronize(c->stream));
  g->host[c->rank].assign(v, v + count);
  if (!barrier(c)) return -1;
  for (int k = 0; k < count; ++k) {
    double a = max ? g->host[0][k] : 0.0;
    for (int q = 0; q < g->n; ++q) {
      const double x = g->host[q][k];
      a = max ? (x > a ? x : a) : a + x;
    }
    v[k] = a;
  }
  return barrier(c) ? 0 : -1;
}

// rank-order gather of variable-size device blocks to root's device buffer
// `recv` (root only; block q lands at offset off[q], off[] known to all ranks)
int comm_gatherv(Ctx *c, int root, const void *send, size_t bytes, void *recv, const size_t *off,
                 const size_t *len) {
  if (!comm_multi(c)) {
    if (bytes && recv != send) BSA_HIP(c, hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, c->stream));
    return 0;
  }
  if (c->comm) {
    BSA_NCCL(c, ncclGroupStart());
    if (c->rank == root) {
      for (int q = 0; q < c->nranks; ++q) {
        if (!len[q]) continue;
        if (q == root)
          BSA_HIP(c, hipMemcpyAsync((char *)recv + off[q], send, len[q], hipMemcpyDeviceToDevice, c->stream));
        else
          BSA_NCCL(c, ncclRecv((char *)recv + off[q], len[q], ncclUint8, q, (ncclComm_t)c->comm, c->stream));
      }
    } else if (bytes) {
      BSA_NCCL(c, ncclSend(send, bytes, ncclUint8, root, (ncclComm_t)c->comm, c->stream));
    }
    BSA_NCCL(c, ncclGroupEnd());
    return 0;
  }
  Group *g = c->group;
  if (publish(c, send, bytes)) return -1;
  if (c->rank == root)
    for (int q = 0; q < g->n; ++q)
      if (len[q])
        BSA_HIP(c, hipMemcpyAsync((char *)recv + off[q], g->slot[q].p, len[q], hipMemcpyDeviceToDevice, c->stream));
  return retire(c);
}

// Halo exchange (bsa_halo.hip): this rank's region for rank q is
// send[soff[q], + slen[q]), rank q's region for this rank lands at
// recv[roff[q], + rlen[q]); peer[q] = where that region starts in rank q's
// send buffer (in-process group).  The lengths are agreed by all ranks (the
// capacity matrix), so every send has its matching receive.
// Region layout agreement of the halo exchange, collective (every rank calls
// it at the same exchange: the trigger is a capacity generation / field count
// that changes on every rank alike).  Each rank contributes what it will send
// to every peer (length, offset in its buffer) and what it expects to receive
// from every peer (length, offset in the peer's buffer); after one host
// all-reduce(max) -- each entry is written by exactly one rank -- every rank
// holds all four R x R matrices and fails, with the same message on every
// rank, if any send disagrees with its receive.  RCCL's grouped send / recv
// with unequal lengths hangs or truncates, so this runs BEFORE ncclGroupStart.
static int halo_check_layout(Ctx *c, const size_t *soff, const size_t *slen, const size_t *rlen,
                             const size_t *peer) {
  const int R = c->nranks, me = c->rank;
  const size_t RR = (size_t)R * R;
  std::vector<double> v(4 * RR, 0.0);  // [send len][send off][expected len][expected off], [sender * R + receiver]
  for (int q = 0; q < R; ++q) {
    if (q == me) continue;
    v[(size_t)me * R + q] = (double)slen[q];
    v[RR + (size_t)me * R + q] = (double)soff[q];
    v[2 * RR + (size_t)q * R + me] = (double)rlen[q];
    v[3 * RR + (size_t)q * R + me] = (double)peer[q];
  }
  if (comm_allreduce_host(c, v.data(), (int)v.size(), true)) return -1;
  for (int s = 0; s < R; ++s)
    for (int q = 0; q < R; ++q) {
      const size_t k = (size_t)s * R + q;
      if (s == q) continue;
      if (v[k] != v[2 * RR + k] || (v[k] != 0.0 && v[RR + k] != v[3 * RR + k]))
        return fail(c, "halo lengths disagree: rank %d sends %.0f B at %.0f, rank %d expects %.0f B at %.0f", s,
                    v[k], v[RR + k], q, v[2 * RR + k], v[3 * RR + k]);
    }
  return 0;
}

int comm_halo(Ctx *c, const void *send, const size_t *soff, const size_t *slen, size_t stot, void *recv,
              const size_t *roff, const size_t *rlen, const size_t *peer) {
  if (!comm_multi(c)) return 0;
  const int R = c->nranks, me = c->rank;
  if (c->halo_chk_gen != c->halo_cap_gen || c->halo_chk_nf != c->halo_fields) {
    if (halo_check_layout(c, soff, slen, rlen, peer)) return -1;
    c->halo_chk_gen = c->halo_cap_gen;
    c->halo_chk_nf = c->halo_fields;
  }
  {
    size_t tx = 0, rx = 0;
    for (int q = 0; q < R; ++q)
      if (q != me) {
        tx += slen[q];
        rx += rlen[q];
      }
    account(c, tx, rx);
  }
  if (c->comm) {
    bool any = false;
    for (int q = 0; q < R; ++q) any = any || (q != me && (slen[q] || rlen[q]));
    if (!any) return 0;
    BSA_NCCL(c, ncclGroupStart());
    for (int q = 0; q < R; ++q) {
      if (q == me) continue;
      if (slen[q])
        BSA_NCCL(c, ncclSend((const char *)send + soff[q], slen[q], ncclUint8, q, (ncclComm_t)c->comm, c->stream));
      if (rlen[q])
        BSA_NCCL(c, ncclRecv((char *)recv + roff[q], rlen[q], ncclUint8, q, (ncclComm_t)c->comm, c->stream));
    }
    BSA_NCCL(c, ncclGroupEnd());
    return 0;
  }
  // In-process group: rank q's region for this rank is copied out of q's
  // published buffer.  RCCL's grouped send / recv needs every send length to
  // equal its receive length (a mismatch hangs or truncates on 8 GPUs), so the
  // lengths and offsets each rank sends with are compared here with what the
  // receiver expects: a disagreement fails loudly on ONE GPU too.
  Group *g = c->group;
  {
    std::lock_guard<std::mutex> lk(g->m);
    g->hlen[me].assign(slen, slen + R);
    g->hlen[me].insert(g->hlen[me].end(), soff, soff + R);
  }
  if (publish(c, send, stot)) return -1;  // (its barrier: every rank's lengths are in place)
  for (int q = 0; q < R; ++q) {
    if (q == me) continue;
    size_t qs = 0, qo = 0;
    {
      std::lock_guard<std::mutex> lk(g->m);
      if (g->hlen[q].size() == (size_t)2 * R) {
        qs = g->hlen[q][(size_t)me];
        qo = g->hlen[q][(size_t)R + me];
      }
    }
    if (qs != rlen[q] || (rlen[q] && qo != peer[q])) {
      fail(c, "halo exchange: rank %d sends %zu B at %zu, rank %d expects %zu B at %zu", q, qs, qo, me, rlen[q],
           peer[q]);
      std::lock_guard<std::mutex> lk(g->m);
      g->broken = true;  // the other ranks fail at their next barrier instead of waiting
      g->cv.notify_all();
      return -1;
    }
    if (rlen[q])
      BSA_HIP(c, hipMemcpyAsync((char *)recv + roff[q], (const char *)g->slot[q].p + peer[q], rlen[q],
                                hipMemcpyDeviceToDevice, c->stream));
  }
  return retire(c);
}

void comm_release(Ctx *c) {
  if (c->comm) {
    ncclCommDestroy((ncclComm_t)c->comm);
    c->comm = nullptr;
  }
  if (c->group) {
    Group *g = c->group;
    bool last = false;
    {
      std::lock_guard<std::mutex> lk(g->m);
      if (g->ctx[c->rank] == c) {
        (void)hipStreamSynchronize(c->stream);
        release(g->slot[c->rank]);
        if (g->pub[c->rank]) (void)hipEventDestroy(g->pub[c->rank]);
        if (g->done[c->rank]) (void)hipEventDestroy(g->done[c->rank]);
        g->pub[c->rank] = g->done[c->rank] = nullptr;
        g->ctx[c->rank] = nullptr;
      }
      last = g->destroy_pending;
      for (int q = 0; q < g->n; ++q) last = last && !g->ctx[q];
    }
    c->group = nullptr;
    if (last) delete g;  // the group was destroyed while this context was its last member
  }
  c->nranks = 1;
  c->rank = 0;
}

}  // namespace bsa

using bsa::Ctx;

struct bsa_group : bsa::Group {};

extern "C" {

int bsa_comm_unique_id(char *id128) {
  if (!id128) return -1;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int bsa_comm_init(bsa_ctx *cc, int nranks, int rank, const char *id128) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!id128 || nranks < 1 || rank < 0 || rank >= nranks) return bsa::fail(c, "bad comm arguments");
  BSA_HIP(c, hipSetDevice(c->device));
  bsa::comm_release(c);
  ncclUniqueId id;
  memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm;
  BSA_NCCL(c, ncclCommInitRank(&comm, nranks, id, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  c->sim_ready = false;  // the row partition changed
  return 0;
}

bsa_group *bsa_group_create(int nranks) {
  if (nranks < 1 || nranks > bsa::kMaxGroup) return nullptr;
  bsa_group *g = new (std::nothrow) bsa_group();
  if (g) g->n = nranks;
  return g;
}

// a group still holding members is freed when its last member leaves
// (bsa_destroy or a new bsa_comm_init*), never under a member's feet
void bsa_group_destroy(bsa_group *g) {
  if (!g) return;
  {
    std::lock_guard<std::mutex> lk(g->m);
    bool members = false;
    for (int q = 0; q < g->n; ++q) members = members || g->ctx[q] != nullptr;
    if (members) {
      g->destroy_pending = true;
      return;
    }
  }
  delete g;
}

int bsa_comm_init_group(bsa_ctx *cc, bsa_group *g, int rank) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (!g || rank < 0 || rank >= g->n) return bsa::fail(c, "bad group arguments");
  BSA_HIP(c, hipSetDevice(c->device));
  bsa::comm_release(c);
  {
    std::lock_guard<std::mutex> lk(g->m);
    if (g->ctx[rank]) return bsa::fail(c, "group rank %d already joined", rank);
    g->ctx[rank] = c;
  }
  hipEvent_t pub = nullptr, done = nullptr;
  BSA_HIP(c, hipEventCreateWithFlags(&pub, hipEventDisableTiming));
  BSA_HIP(c, hipEventCreateWithFlags(&done, hipEventDisableTiming));
  BSA_HIP(c, hipEventRecord(pub, c->stream));
  BSA_HIP(c, hipEventRecord(done, c->stream));
  {  // published under the lock (publish() of a rank already running reads them)
    std::lock_guard<std::mutex> lk(g->m);
    g->pub[rank] = pub;
    g->done[rank] = done;
  }
  c->group = g;
  c->nranks = g->n;
  c->rank = rank;
  c->sim_ready = false;
  return 0;
}

// C2: per-rank (P, L, rows) of the last detect, all ranks
static int gather_layout(Ctx *c, std::vector<int64_t> &cnt) {
  if (bsa::sim_adopt_pairs(c)) return -1;
  if (!c->have_pairs) return bsa::fail(c, "no detect results to gather");
  std::vector<double> v((size_t)3 * c->nranks, 0.0);
  v[3 * c->rank + 0] = (double)c->last_conf;
  v[3 * c->rank + 1] = (double)c->last_los;
  v[3 * c->rank + 2] = (double)(c->last_re - c->last_rb);
  if (bsa::comm_allreduce_host(c, v.data(), (int)v.size(), false)) return -1;
  cnt.resize(v.size());
  for (size_t k = 0; k < v.size(); ++k) cnt[k] = (int64_t)v[k];
  return 0;
}

// one rank's packed block: ci cj (P int32) | payload 5 x P doubles | li lj (L int32) | inconf (R) | tcpamax (R)
static size_t al8(size_t b) { return (b + 7) & ~size_t(7); }
static size_t block_bytes(int64_t P, int64_t L, int64_t R) {
  return al8((size_t)P * 8) + (size_t)P * 40 + al8((size_t)L * 8) + al8((size_t)R) + (size_t)R * 8;
}

int bsa_gather_counts(bsa_ctx *cc, int64_t *totals3) {
  Ctx *c = (Ctx *)cc;
  if (!c || !totals3) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<int64_t> cnt;
  if (gather_layout(c, cnt)) return -1;
  totals3[0] = totals3[1] = totals3[2] = 0;
  for (int q = 0; q < c->nranks; ++q)
    for (int k = 0; k < 3; ++k) totals3[k] += cnt[3 * q + k];
  return 0;
}

int bsa_gather_pairs(bsa_ctx *cc, int root, const bsa_pairs_out *out) {
  Ctx *c = (Ctx *)cc;
  if (!c) return -1;
  if (root < 0 || root >= c->nranks) return bsa::fail(c, "bad root rank %d", root);
  if (c->rank == root && !out) return bsa::fail(c, "NULL output on the root rank");
  BSA_HIP(c, hipSetDevice(c->device));
  std::vector<int64_t> cnt;
  if (gather_layout(c, cnt)) return -1;
  const int nr = c->nranks;
  std::vector<size_t> off(nr), len(nr);
  size_t total = 0;
  for (int q = 0; q < nr; ++q) {
    off[q] = total;
    len[q] = block_bytes(cnt[3 * q], cnt[3 * q + 1], cnt[3 * q + 2]);
    total += len[q];
  }
  // pack this rank's block (device to device, stream-ordered after the detect)
  const int64_t P = c->last_conf, L = c->last_los, R = c->last_re - c->last_rb;
  if (!bsa::ensure(c, c->pg_send, len[c->rank], "pair gather block")) return -1;
  char *b = (char *)c->pg_send.p;
  hipStream_t s = c->stream;
  auto d2d = [&](size_t at, const void *src, size_t bytes) -> int {
    if (bytes) BSA_HIP(c, hipMemcpyAsync(b + at, src, bytes, hipMemcpyDeviceToDevice, s));
    return 0;
  };
  size_t at = 0;
  if (d2d(at, c->out_ci.p, (size_t)P * 4) || d2d(at + (size_t)P * 4, c->out_cj.p, (size_t)P * 4)) return -1;
  at += al8((size_t)P * 8);
  if (d2d(at, c->out_pay.p, (size_t)P * 40)) return -1;
  at += (size_t)P * 40;
  if (d2d(at, c->out_li.p, (size_t)L * 4) || d2d(at + (size_t)L * 4, c->out_lj.p, (size_t)L * 4)) return -1;
  at += al8((size_t)L * 8);
  if (d2d(at, c->inconf.p, (size_t)R)) return -1;
  at += al8((size_t)R);
  if (d2d(at, c->tcpamax.p, (size_t)R * 8)) return -1;
  if (c->rank == root && !bsa::ensure(c, c->pg_recv, total, "pair gather")) return -1;
  if (bsa::comm_gatherv(c, root, c->pg_send.p, len[c->rank], c->rank == root ? c->pg_recv.p : nullptr, off.data(),
                        len.data()))
    return -1;
  if (c->rank != root) return 0;
  std::vector<char> h(total);
  if (total) BSA_HIP(c, hipMemcpyAsync(h.data(), c->pg_recv.p, total, hipMemcpyDeviceToHost, s));
  BSA_HIP(c, hipStreamSynchronize(s));
  // concatenate in rank order: the ranks' rows are consecutive home ranges,
  // so this is all rows in home order; home rows -> aircraft indices in
  // global row-major order (home_pairs_to_ids)
  int64_t Pt = 0, Lt = 0, Rt = 0;
  for (int q = 0; q < nr; ++q) {
    Pt += cnt[3 * q];
    Lt += cnt[3 * q + 1];
    Rt += cnt[3 * q + 2];
  }
  bsa::HostPairs hp;
  hp.ci.resize((size_t)Pt);
  hp.cj.resize((size_t)Pt);
  hp.pay.resize((size_t)Pt * 5);
  hp.li.resize((size_t)Lt);
  hp.lj.resize((size_t)Lt);
  hp.inconf.resize((size_t)Rt);
  hp.tcpamax.resize((size_t)Rt);
  int64_t pc = 0, pl = 0, pr = 0;
  for (int q = 0; q < nr; ++q) {
    const int64_t Pq = cnt[3 * q], Lq = cnt[3 * q + 1], Rq = cnt[3 * q + 2];
    const char *blk = h.data() + off[q];
    auto put = [](void *dst, int64_t at_elems, size_t esz, const char *src, int64_t n) {
      if (n) memcpy((char *)dst + (size_t)at_elems * esz, src, (size_t)n * esz);
    };
    put(hp.ci.data(), pc, 4, blk, Pq);
    put(hp.cj.data(), pc, 4, blk + (size_t)Pq * 4, Pq);
    const char *pay = blk + al8((size_t)Pq * 8);
    for (int f = 0; f < 5; ++f) put(hp.pay.data() + (size_t)f * Pt, pc, 8, pay + (size_t)f * Pq * 8, Pq);
    const char *lp = pay + (size_t)Pq * 40;
    put(hp.li.data(), pl, 4, lp, Lq);
    put(hp.lj.data(), pl, 4, lp + (size_t)Lq * 4, Lq);
    const char *rp = lp + al8((size_t)Lq * 8);
    put(hp.inconf.data(), pr, 1, rp, Rq);
    put(hp.tcpamax.data(), pr, 8, rp + al8((size_t)Rq), Rq);
    pc += Pq;
    pl += Lq;
    pr += Rq;
  }
  if (c->last_home) bsa::home_pairs_to_ids(c, 0, hp);
  auto out_put = [](void *dst, const void *src, size_t bytes) {
    if (dst && bytes) memcpy(dst, src, bytes);
  };
  out_put(out->ci, hp.ci.data(), (size_t)Pt * 4);
  out_put(out->cj, hp.cj.data(), (size_t)Pt * 4);
  double *dst5[5] = {out->qdr, out->dist, out->tcpa, out->tinconf, out->dcpa};
  for (int f = 0; f < 5; ++f) out_put(dst5[f], hp.pay.data() + (size_t)f * Pt, (size_t)Pt * 8);
  out_put(out->li, hp.li.data(), (size_t)Lt * 4);
  out_put(out->lj, hp.lj.data(), (size_t)Lt * 4);
  out_put(out->inconf, hp.inconf.data(), (size_t)Rt);
  out_put(out->tcpamax, hp.tcpamax.data(), (size_t)Rt * 8);
  return 0;
}

int bsa_comm_allreduce_max(bsa_ctx *cc, double *values, int count) {
  Ctx *c = (Ctx *)cc;
  if (!c || (!values && count > 0)) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::comm_allreduce_host(c, values, count, true);
}

int bsa_comm_allreduce_sum(bsa_ctx *cc, double *values, int count) {
  Ctx *c = (Ctx *)cc;
  if (!c || (!values && count > 0)) return -1;
  BSA_HIP(c, hipSetDevice(c->device));
  return bsa::comm_allreduce_host(c, values, count, false);
}

int bsa_comm_info(bsa_ctx *cc, int *info4) {
  Ctx *c = (Ctx *)cc;
  if (!c || !info4) return -1;
  info4[0] = 0;
  info4[1] = c->nranks;
  info4[2] = c->rank;
  info4[3] = c->device;
  if (c->comm) {  // RCCL's own view of the communicator
    int n = 0, r = 0, d = 0;
    BSA_NCCL(c, ncclCommCount((ncclComm_t)c->comm, &n));
    BSA_NCCL(c, ncclCommUserRank((ncclComm_t)c->comm, &r));
    BSA_NCCL(c, ncclCommCuDevice((ncclComm_t)c->comm, &d));
    info4[0] = 1;
    info4[1] = n;
    info4[2] = r;
    info4[3] = d;
  } else if (c->group) {
    info4[0] = 2;
  }
  return 0;
}

}  // extern "C"
