// RCCL communicator and the hash-aggregate exchange in the C ABI ("qe_agg_exchange(comm,
// partial) -> partial (RCCL)"): the multi-GPU form of main()'s partial -> final merge
// (Main.kt:1309-1325) for hosts without torch.distributed — a JNI caller creates one qe_comm per
// GPU from a unique id it broadcasts itself (rank 0's qe_comm_unique_id), then every rank calls
// qe_hashagg_exchange after its partial aggregation.
//
// The exchange runs entirely on the ctx stream: export of fixed-capacity slots (no host wait
// before it, qe_hashagg_export_slots), ONE grouped send/recv of equal slots between every pair of
// ranks over xGMI, and the slot import with its single read-back (qe_hashagg_import_slots). When a
// sender's partition exceeded the slot capacity — every rank sees the same verdict in the slot
// headers — all ranks fall back together to a variable-size exchange: per-destination counts,
// then the records.
//
// RCCL is loaded at run time (dlopen of librccl.so.1, RTLD_LOCAL), so the library keeps no link
// dependency on it and shares the process's copy when a framework has loaded one already.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "qe_internal.hpp"

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      const char* e = dlerror();
      r.why = e ? e : "librccl.so.1 not found";
      return;
    }
    bool all = true;
    auto sym = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      all = all && fp != nullptr;
    };
    sym(r.get_unique_id, "ncclGetUniqueId");
    sym(r.comm_init_rank, "ncclCommInitRank");
    sym(r.comm_destroy, "ncclCommDestroy");
    sym(r.send, "ncclSend");
    sym(r.recv, "ncclRecv");
    sym(r.group_start, "ncclGroupStart");
    sym(r.group_end, "ncclGroupEnd");
    sym(r.error_string, "ncclGetErrorString");
    r.ok = all;
    if (!all) r.why = "librccl is missing an entry point";
  });
  return r;
}

#define QE_NCCL(call)                                                                               \
  do {                                                                                              \
    const ncclResult_t qe_r_ = (call);                                                              \
    if (qe_r_ != ncclSuccess)                                                                       \
      return ::qe::fail(QE_ERR_COMM, "%s failed: %s", #call, rccl().error_string(qe_r_));           \
  } while (0)

}  // namespace

// In-process transport (qe_comm_create_loopback): the ranks are threads of one process, each with
// its own qe_ctx; a grouped send/recv becomes "publish my send buffers, wait for every rank, copy
// what the peers address to me, wait again". The hash-aggregate exchange above it is the same code
// as over RCCL — what a single-GPU box can run of the multi-rank path (RCCL refuses two ranks on
// one device).
struct qe_loop_hub {
  int32_t world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int32_t arrived = 0;
  uint64_t generation = 0;
  std::vector<const uint8_t*> send;
  std::vector<const size_t*> soff, sbytes;
  std::vector<int> failed;
  void barrier() {
    std::unique_lock<std::mutex> g(mu);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(g, [&] { return generation != gen; });
    }
  }
};

struct qe_comm {
  qe_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  qe_loop_hub* hub = nullptr;  // in-process transport instead of RCCL
  int32_t world = 0, rank = 0;
  uint8_t* buf = nullptr;  // send | recv slots (device), grown as needed
  size_t buf_bytes = 0;
};

using namespace qe;

namespace {

int comm_buffer(qe_comm* c, size_t bytes) {
  if (bytes <= c->buf_bytes) return QE_OK;
  dev_free(c->ctx, c->buf);
  c->buf = nullptr;
  c->buf_bytes = 0;
  QE_TRY(dev_alloc(c->ctx, bytes, (void**)&c->buf));
  c->buf_bytes = bytes;
  return QE_OK;
}

// Grouped point-to-point: rank p gets send + soff[p] (sbytes[p] bytes) into recv + roff[p].
int exchange_bytes(qe_comm* c, const uint8_t* send, const size_t* soff, const size_t* sbytes, uint8_t* recv,
                   const size_t* roff, const size_t* rbytes) {
  if (c->hub) {  // in-process ranks: publish, wait, copy what the peers address to this rank, wait
    qe_loop_hub* h = c->hub;
    // a rank that fails still passes both barriers (its peers would wait forever otherwise) and
    // publishes the failure, so that every rank skips the copies and reports it
    int st = ctx_sync(c->ctx);  // the send buffers are complete
    h->send[c->rank] = send;
    h->soff[c->rank] = soff;
    h->sbytes[c->rank] = sbytes;
    h->failed[c->rank] = st != QE_OK;
    h->barrier();
    for (int p = 0; p < c->world && st == QE_OK; ++p)
      if (h->failed[p]) st = fail(QE_ERR_COMM, "loopback exchange: rank %d failed before the exchange", p);
    for (int p = 0; p < c->world && st == QE_OK; ++p) {
      if (h->sbytes[p][c->rank] != rbytes[p])
        st = fail(QE_ERR_COMM, "loopback exchange: rank %d sends %zu bytes to rank %d, which expects %zu", p,
                  h->sbytes[p][c->rank], c->rank, rbytes[p]);
      else if (rbytes[p] && hipMemcpyAsync(recv + roff[p], h->send[p] + h->soff[p][c->rank], rbytes[p],
                                           hipMemcpyDeviceToDevice, c->ctx->stream) != hipSuccess)
        st = fail(QE_ERR_DEVICE, "loopback exchange: copy from rank %d failed", p);
    }
    if (st == QE_OK) st = ctx_sync(c->ctx);
    h->barrier();  // every rank has copied out of every send buffer before any is reused
    return st;
  }
  const Rccl& R = rccl();
  QE_NCCL(R.group_start());
  ncclResult_t r = ncclSuccess;
  for (int p = 0; p < c->world && r == ncclSuccess; ++p) {
    if (sbytes[p]) r = R.send(send + soff[p], sbytes[p], ncclUint8, p, c->comm, c->ctx->stream);
    if (r == ncclSuccess && rbytes[p]) r = R.recv(recv + roff[p], rbytes[p], ncclUint8, p, c->comm, c->ctx->stream);
  }
  const ncclResult_t e = R.group_end();  // the group is closed whatever failed inside it
  QE_NCCL(r);
  QE_NCCL(e);
  return QE_OK;
}

// Dictionary-keyed partials (K:1336's VendorID): blocks by key content. One all-to-all of the block
// sizes, then the blocks; the owner re-encodes the keys into its own dictionaries.
int exchange_keyed(qe_comm* c, qe_hashagg* partial, qe_hashagg* owner, int64_t* nrecords) {
  const int world = c->world;
  std::vector<int64_t> sb(world), rb(world);
  QE_TRY(qe_hashagg_export_keyed_sizes(partial, world, sb.data()));
  QE_TRY(comm_buffer(c, (size_t)2 * world * 8));
  int64_t* dsz = (int64_t*)c->buf;
  QE_HIP(hipMemcpyAsync(dsz, sb.data(), (size_t)world * 8, hipMemcpyHostToDevice, c->ctx->stream));
  std::vector<size_t> o8(world), l8(world, 8);
  for (int p = 0; p < world; ++p) o8[p] = (size_t)p * 8;
  QE_TRY(exchange_bytes(c, (const uint8_t*)dsz, o8.data(), l8.data(), (uint8_t*)(dsz + world), o8.data(), l8.data()));
  QE_HIP(hipMemcpyAsync(rb.data(), dsz + world, (size_t)world * 8, hipMemcpyDeviceToHost, c->ctx->stream));
  QE_TRY(ctx_sync(c->ctx));
  std::vector<size_t> so(world), sl(world), ro(world), rl(world);
  size_t a = 0, b = 0;
  for (int p = 0; p < world; ++p) {
    so[p] = a;
    sl[p] = (size_t)sb[p];
    a += sl[p];
    ro[p] = b;
    rl[p] = (size_t)rb[p];
    b += rl[p];
  }
  QE_TRY(comm_buffer(c, std::max<size_t>(a + b, 8)));
  uint8_t* send = c->buf;
  uint8_t* recv = c->buf + a;
  QE_TRY(qe_hashagg_export_keyed(partial, world, send));
  QE_TRY(exchange_bytes(c, send, so.data(), sl.data(), recv, ro.data(), rl.data()));
  QE_TRY(qe_hashagg_import_keyed(owner, recv, world, rb.data()));
  if (nrecords) {  // records this rank merged: the received blocks' counts (header word 1)
    std::vector<int64_t> nrec(world, 0);
    for (int p = 0; p < world; ++p)
      if (rb[p]) QE_HIP(hipMemcpyAsync(&nrec[p], recv + ro[p] + 8, 8, hipMemcpyDeviceToHost, c->ctx->stream));
    QE_TRY(ctx_sync(c->ctx));
    int64_t n = 0;
    for (int64_t x : nrec) n += x;
    *nrecords = n;
  }
  return QE_OK;
}

}  // namespace

extern "C" {

int qe_comm_unique_id(void* id) {
  QE_CHECK(id, QE_ERR_INVALID_ARG, "null id");
  const Rccl& R = rccl();
  QE_CHECK(R.ok, QE_ERR_COMM, "RCCL unavailable: %s", R.why.c_str());
  static_assert(sizeof(ncclUniqueId) == QE_COMM_ID_BYTES, "unique id size");
  ncclUniqueId u;
  QE_NCCL(R.get_unique_id(&u));
  memcpy(id, &u, sizeof u);
  return QE_OK;
}

int qe_comm_create(qe_ctx* ctx, int32_t world, int32_t rank, const void* id, qe_comm** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out && id && world >= 1 && rank >= 0 && rank < world, QE_ERR_INVALID_ARG, "bad arguments");
  const Rccl& R = rccl();
  QE_CHECK(R.ok, QE_ERR_COMM, "RCCL unavailable: %s", R.why.c_str());
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  ncclComm_t comm = nullptr;
  QE_NCCL(R.comm_init_rank(&comm, world, u, rank));  // collective: every rank of the id calls it
  qe_comm* c = new qe_comm();
  c->ctx = ctx;
  c->comm = comm;
  c->world = world;
  c->rank = rank;
  *out = c;
  return QE_OK;
}

int qe_comm_destroy(qe_comm* c) {
  if (!c) return QE_OK;
  (void)hipSetDevice(c->ctx->device);
  (void)hipStreamSynchronize(c->ctx->stream);
  dev_free(c->ctx, c->buf);
  if (c->comm) (void)rccl().comm_destroy(c->comm);
  delete c;
  return QE_OK;
}

int qe_comm_loopback_hub_create(int32_t world, void** hub) {
  QE_CHECK(hub && world >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  qe_loop_hub* h = new qe_loop_hub();
  h->world = world;
  h->send.assign(world, nullptr);
  h->soff.assign(world, nullptr);
  h->sbytes.assign(world, nullptr);
  h->failed.assign(world, 0);
  *hub = h;
  return QE_OK;
}

int qe_comm_loopback_hub_destroy(void* hub) {
  delete (qe_loop_hub*)hub;
  return QE_OK;
}

int qe_comm_create_loopback(qe_ctx* ctx, int32_t world, int32_t rank, void* hub, qe_comm** out) {
  QE_TRY(ctx_enter(ctx));
  qe_loop_hub* h = (qe_loop_hub*)hub;
  QE_CHECK(out && h && world == h->world && rank >= 0 && rank < world, QE_ERR_INVALID_ARG, "bad arguments");
  qe_comm* c = new qe_comm();
  c->ctx = ctx;
  c->hub = h;
  c->world = world;
  c->rank = rank;
  *out = c;
  return QE_OK;
}

int qe_hashagg_slot_capacity(qe_hashagg* h, int32_t world, int64_t* cap) {
  QE_CHECK(h && cap && world >= 1, QE_ERR_INVALID_ARG, "bad arguments");
  // the create-time expected groups spread over the ranks with headroom: 1.5x an even share plus
  // 32, at most the expected groups. It depends on nothing a rank's own data changes, so every
  // rank computes the same slot size (the all-to-all's slots must be equal).
  int64_t eg = 0;
  QE_TRY(hashagg_expected_groups(h, &eg));
  eg = std::max<int64_t>(eg, 1);
  *cap = std::min<int64_t>(eg, (3 * eg + 2 * world - 1) / (2 * world) + 32);
  return QE_OK;
}

int qe_hashagg_exchange(qe_comm* c, qe_hashagg* partial, qe_hashagg* owner, int64_t slot_records,
                        int64_t* nrecords) {
  QE_CHECK(c && partial && owner, QE_ERR_INVALID_ARG, "null argument");
  QE_TRY(ctx_enter(c->ctx));
  const int world = c->world;
  int64_t rb = 0;
  QE_TRY(qe_hashagg_record_bytes(partial, &rb));
  QE_CHECK(hashagg_ctx(partial) == c->ctx && hashagg_ctx(owner) == c->ctx, QE_ERR_INVALID_ARG,
           "partial, owner and communicator must share one qe_ctx (one stream)");
  if (keyed_dict(hashagg_info(partial).keyed) || keyed_dict(hashagg_info(owner).keyed))
    return exchange_keyed(c, partial, owner, nrecords);
  int64_t cap = slot_records;
  if (cap <= 0) QE_TRY(qe_hashagg_slot_capacity(partial, world, &cap));
  const size_t slot_bytes = (size_t)QE_SLOT_HEADER + (size_t)cap * (size_t)rb;
  QE_TRY(comm_buffer(c, 2 * (size_t)world * slot_bytes));
  uint8_t* send = c->buf;
  uint8_t* recv = c->buf + (size_t)world * slot_bytes;
  QE_TRY(qe_hashagg_export_slots(partial, world, cap, send));
  std::vector<size_t> off(world), len(world, slot_bytes);
  for (int p = 0; p < world; ++p) off[p] = (size_t)p * slot_bytes;
  QE_TRY(exchange_bytes(c, send, off.data(), len.data(), recv, off.data(), len.data()));
  int64_t mx = 0, n = 0;
  QE_TRY(qe_hashagg_import_slots(owner, recv, world, cap, &mx, &n));
  if (mx <= cap) {
    if (nrecords) *nrecords = n;
    return QE_OK;
  }
  // some partition did not fit a slot (same verdict on every rank): counts, then the records
  std::vector<int64_t> counts(world);
  QE_TRY(qe_hashagg_export_counts(partial, world, counts.data()));
  int64_t total = 0;
  for (int64_t x : counts) total += x;
  QE_TRY(comm_buffer(c, (size_t)2 * world * 8 + (size_t)std::max<int64_t>(total, 1) * rb));
  int64_t* dcnt = (int64_t*)c->buf;
  QE_HIP(hipMemcpyAsync(dcnt, counts.data(), (size_t)world * 8, hipMemcpyHostToDevice, c->ctx->stream));
  std::vector<size_t> o8(world), l8(world, 8);
  for (int p = 0; p < world; ++p) o8[p] = (size_t)p * 8;
  QE_TRY(exchange_bytes(c, (const uint8_t*)dcnt, o8.data(), l8.data(), (uint8_t*)(dcnt + world), o8.data(),
                        l8.data()));
  std::vector<int64_t> rcounts(world);
  QE_HIP(hipMemcpyAsync(rcounts.data(), dcnt + world, (size_t)world * 8, hipMemcpyDeviceToHost, c->ctx->stream));
  QE_TRY(ctx_sync(c->ctx));
  int64_t rtotal = 0;
  for (int64_t x : rcounts) rtotal += x;
  // layout: [counts | recv counts | send records | recv records]
  const size_t head = (size_t)2 * world * 8;
  QE_TRY(comm_buffer(c, head + (size_t)(std::max<int64_t>(total, 1) + std::max<int64_t>(rtotal, 1)) * rb));
  uint8_t* srec = c->buf + head;
  uint8_t* rrec = srec + (size_t)std::max<int64_t>(total, 1) * rb;
  QE_TRY(qe_hashagg_export(partial, world, srec));  // partition-major, counts as above
  std::vector<size_t> so(world), sl(world), ro(world), rl(world);
  size_t a = 0, b = 0;
  for (int p = 0; p < world; ++p) {
    so[p] = a;
    sl[p] = (size_t)counts[p] * rb;
    a += sl[p];
    ro[p] = b;
    rl[p] = (size_t)rcounts[p] * rb;
    b += rl[p];
  }
  QE_TRY(exchange_bytes(c, srec, so.data(), sl.data(), rrec, ro.data(), rl.data()));
  QE_TRY(qe_hashagg_import(owner, rrec, rtotal));
  if (nrecords) *nrecords = rtotal;
  return QE_OK;
}

}  // extern "C"
