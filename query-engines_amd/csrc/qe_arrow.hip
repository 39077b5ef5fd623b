// Drop-in boundary at batch level: Arrow C Data Interface in and out.
//
// The reference's columns are Arrow Java vectors (ArrowFieldVector, Main.kt:176-202; built by
// ArrowVectorBuilder K:481-511 into VectorSchemaRoot K:635-650). Arrow Java exports/imports a
// VectorSchemaRoot as a struct ArrowArray + ArrowSchema (org.apache.arrow.c.Data), so a JNI shim
// hands this library exactly these structs:
//   qe_batch_import         host struct array -> device batch (H2D through pinned staging, 8 host
//                           threads with double buffers; sliced arrays / unaligned validity rebased)
//   qe_batch_import_device  ArrowDeviceArray already in HBM (ARROW_DEVICE_ROCM) -> zero-copy view
//   qe_batch_export         device columns -> host struct array (release frees the host copy)
// Types: l int64, g float64, u utf8 (U large-utf8 when it fits int32 offsets), i int32,
// C uint8, tdD date32, b bool. Anything else is QE_ERR_UNSUPPORTED (cf. K:195).
#include <errno.h>
#include <fcntl.h>
#include <stdlib.h>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "qe_internal.hpp"

struct qe_batch {
  qe_ctx* ctx = nullptr;
  int64_t length = 0;
  std::vector<qe_column> cols;
  std::vector<std::string> names;
  void* device_block = nullptr;  // owned device memory (host imports); null for device views
};

namespace qe {
namespace {

// Parallel staged H2D for a whole batch: the copies are cut into chunks and dealt round-robin to
// up to 8 host threads; each thread memcpys a chunk into its own pinned half (two halves per
// thread, an event per half) and enqueues the DMA on the ctx stream. One host thread's memcpy into
// pinned memory (~28 GB/s measured) is what limits a single-threaded stager below the link (~57 GB/s).
struct H2DJob {
  uint8_t* dst;
  const uint8_t* src;  // host bytes, or null: read from file `fd` at `foff`
  size_t n;
  int fd = -1;
  int64_t foff = 0;
};
// Staging chunk (QE_STAGE_MB, default 16): per-chunk DMA + event costs dominate small chunks.
// 2.4 GB import measured: 2 MiB 40.0 GB/s, 4 MiB 46.4, 8 MiB 50.7, 16 MiB 53.3, 32 MiB 53.9,
// 64 MiB 53.3; 8 batches of 300 MB: 16 MiB best (53.0 ms; 32 MiB 60.1 ms: pipeline fill).
size_t stage_chunk() {
  static const size_t c = [] {
    const char* e = getenv("QE_STAGE_MB");
    const long v = e && *e ? atol(e) : 16;
    return (size_t)(v >= 1 && v <= 64 ? v : 16) << 20;
  }();
  return c;
}
constexpr int PTHREADS = 8;

// Persistent staging workers (creating 7 threads per import cost ~0.3 ms). Calls from several
// host threads share them: each call queues its tasks and runs its first task inline.
class StagePool {
 public:
  explicit StagePool(int n) {
    for (int i = 0; i < n; ++i) std::thread([this] { loop(); }).detach();
  }
  void run(std::vector<std::function<void()>>& tasks) {
    if (tasks.empty()) return;
    std::mutex dm;
    std::condition_variable dcv;
    size_t left = tasks.size() - 1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (size_t i = 1; i < tasks.size(); ++i)
        q_.push_back([&, i] {
          tasks[i]();
          std::lock_guard<std::mutex> l2(dm);
          if (--left == 0) dcv.notify_one();
        });
    }
    cv_.notify_all();
    tasks[0]();
    std::unique_lock<std::mutex> l2(dm);
    dcv.wait(l2, [&] { return left == 0; });
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [this] { return !q_.empty(); });
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
};

StagePool& stage_pool() {
  static StagePool* p = new StagePool(PTHREADS - 1);  // never destroyed: idle workers at exit
  return *p;
}

int parallel_h2d(qe_ctx* ctx, const std::vector<H2DJob>& jobs) {
  std::vector<H2DJob> chunks;
  const size_t PSTAGE = stage_chunk();
  // The first chunk of every thread is small: the link idles until some thread has filled its first
  // pinned half, so a 16 MiB first round (~2-3 ms of memcpy / pread per thread) would be pure
  // pipeline fill; later chunks are large (per-chunk DMA + event costs).
  const size_t RAMP = std::min<size_t>(PSTAGE, (size_t)2 << 20);
  for (const H2DJob& j : jobs)
    for (size_t o = 0; o < j.n;) {
      const size_t c = std::min(chunks.size() < (size_t)PTHREADS ? RAMP : PSTAGE, j.n - o);
      chunks.push_back({j.dst + o, j.src ? j.src + o : nullptr, c, j.fd, j.foff + (int64_t)o});
      o += c;
    }
  if (chunks.empty()) return QE_OK;
  const int T = (int)std::min<size_t>(PTHREADS, chunks.size());
  void* pin;
  QE_TRY(ctx_pinned(ctx, (size_t)T * 2 * PSTAGE, &pin));
  std::vector<int> rc((size_t)T, QE_OK);
  std::vector<std::string> err((size_t)T);
  auto work = [&](int t) {
    if (hipSetDevice(ctx->device) != hipSuccess) {
      rc[(size_t)t] = QE_ERR_DEVICE;
      return;
    }
    uint8_t* half[2] = {(uint8_t*)pin + (size_t)(2 * t) * PSTAGE, (uint8_t*)pin + (size_t)(2 * t + 1) * PSTAGE};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    int cur = 0;
    for (int h = 0; h < 2; ++h)
      if (hipEventCreateWithFlags(&ev[h], hipEventDisableTiming) != hipSuccess) rc[(size_t)t] = QE_ERR_DEVICE;
    for (size_t j = (size_t)t; j < chunks.size() && rc[(size_t)t] == QE_OK; j += (size_t)T) {
      if (busy[cur] && hipEventSynchronize(ev[cur]) != hipSuccess) rc[(size_t)t] = QE_ERR_DEVICE;
      if (chunks[j].src) {
        memcpy(half[cur], chunks[j].src, chunks[j].n);
      } else {  // straight from the file into pinned memory: no mapping, no page faults in this process
        size_t got = 0;
        while (got < chunks[j].n) {
          const ssize_t r = pread(chunks[j].fd, half[cur] + got, chunks[j].n - got, (off_t)(chunks[j].foff + got));
          if (r <= 0) {
            if (r < 0 && errno == EINTR) continue;
            rc[(size_t)t] = QE_ERR_INVALID_ARG;
            err[(size_t)t] = r < 0 ? strerror(errno) : "file shorter than requested";
            break;
          }
          got += (size_t)r;
        }
        if (rc[(size_t)t] != QE_OK) break;
      }
      if (hipMemcpyAsync(chunks[j].dst, half[cur], chunks[j].n, hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
          hipEventRecord(ev[cur], ctx->stream) != hipSuccess)
        rc[(size_t)t] = QE_ERR_DEVICE;
      busy[cur] = true;
      cur ^= 1;
    }
    for (int h = 0; h < 2; ++h) {
      if (busy[h]) (void)hipEventSynchronize(ev[h]);
      if (ev[h]) (void)hipEventDestroy(ev[h]);
    }
  };
  std::vector<std::function<void()>> tasks;
  for (int t = 0; t < T; ++t) tasks.push_back([&work, t] { work(t); });
  stage_pool().run(tasks);
  for (int t = 0; t < T; ++t)
    if (rc[(size_t)t] != QE_OK) {
      (void)ctx_sync(ctx);  // the other threads' DMAs out of the staging buffers
      if (rc[(size_t)t] == QE_ERR_INVALID_ARG) return fail(QE_ERR_INVALID_ARG, "file read failed: %s", err[(size_t)t].c_str());
      return fail(QE_ERR_DEVICE, "host-to-device staging failed");
    }
  QE_TRY(ctx_sync(ctx));
  return QE_OK;
}

// Arrow format string -> QE type (0 = unsupported).
int32_t type_of_format(const char* f) {
  if (!f) return 0;
  if (!strcmp(f, "l")) return QE_TYPE_INT64;
  if (!strcmp(f, "g")) return QE_TYPE_FLOAT64;
  if (!strcmp(f, "u") || !strcmp(f, "U")) return QE_TYPE_UTF8;
  if (!strcmp(f, "i")) return QE_TYPE_INT32;
  if (!strcmp(f, "C")) return QE_TYPE_UINT8;
  if (!strcmp(f, "tdD")) return QE_TYPE_DATE32;
  if (!strcmp(f, "b")) return QE_TYPE_BOOL;
  return 0;
}

const char* format_of_type(int32_t t) {
  switch (t) {
    case QE_TYPE_INT64: return "l";
    case QE_TYPE_FLOAT64: return "g";
    case QE_TYPE_UTF8: return "u";
    case QE_TYPE_INT32: return "i";
    case QE_TYPE_UINT8: return "C";
    case QE_TYPE_DATE32: return "tdD";
    case QE_TYPE_BOOL: return "b";
    default: return nullptr;
  }
}

inline size_t bitmap_words_bytes(int64_t n) { return (size_t)div_up((uint64_t)(n > 0 ? n : 1), 32) * 4; }
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// bits [off, off+n) of src -> dst (LSB-first), padded with zeros to whole words.
void copy_bits(uint8_t* dst, const uint8_t* src, int64_t off, int64_t n, size_t dst_bytes) {
  memset(dst, 0, dst_bytes);
  if ((off & 7) == 0) {
    memcpy(dst, src + off / 8, (size_t)div_up((uint64_t)n, 8));
    if (n & 7) dst[n / 8] &= (uint8_t)((1u << (n & 7)) - 1);
    return;
  }
  for (int64_t i = 0; i < n; ++i) {
    const int64_t j = off + i;
    if ((src[j >> 3] >> (j & 7)) & 1) dst[i >> 3] |= (uint8_t)(1u << (i & 7));
  }
}

struct ColPlan {
  int32_t type;
  int64_t off, len;
  const uint8_t* validity;  // host (null = all valid)
  const void* values;
  const void* offsets;      // utf8
  bool large;               // 'U'
  int64_t byte0, nbytes;    // utf8 byte range
  size_t o_valid, o_values, o_offs, sz_valid, sz_values, sz_offs;
};

int plan_column(const ArrowSchema* s, const ArrowArray* a, int64_t parent_off, int64_t len, ColPlan* p) {
  p->type = type_of_format(s->format);
  QE_CHECK(p->type != 0, QE_ERR_UNSUPPORTED, "Arrow format '%s' is not supported (field %s)",
           s->format ? s->format : "?", s->name ? s->name : "?");
  QE_CHECK(a->length >= parent_off + len || a->length >= len, QE_ERR_INVALID_ARG, "child array shorter than batch");
  p->off = a->offset + parent_off;
  p->len = len;
  p->large = s->format && !strcmp(s->format, "U");
  QE_CHECK(a->n_buffers >= (p->type == QE_TYPE_UTF8 ? 3 : 2), QE_ERR_INVALID_ARG, "Arrow array has %lld buffers",
           (long long)a->n_buffers);
  p->validity = (a->null_count != 0) ? (const uint8_t*)a->buffers[0] : nullptr;
  p->values = p->type == QE_TYPE_UTF8 ? a->buffers[2] : a->buffers[1];
  p->offsets = p->type == QE_TYPE_UTF8 ? a->buffers[1] : nullptr;
  p->sz_valid = p->validity ? bitmap_words_bytes(len) : 0;
  p->byte0 = p->nbytes = 0;
  p->sz_offs = 0;
  if (p->type == QE_TYPE_UTF8) {
    if (p->large) {
      const int64_t* o = (const int64_t*)p->offsets;
      p->byte0 = o[p->off];
      p->nbytes = o[p->off + len] - p->byte0;
    } else {
      const int32_t* o = (const int32_t*)p->offsets;
      p->byte0 = o[p->off];
      p->nbytes = (int64_t)o[p->off + len] - p->byte0;
    }
    QE_CHECK(p->nbytes < (1ll << 31), QE_ERR_CAPACITY, "utf8 column over 2^31 bytes");
    p->sz_offs = (size_t)(len + 1) * 4;
    p->sz_values = (size_t)(p->nbytes > 0 ? p->nbytes : 1);
  } else if (p->type == QE_TYPE_BOOL) {
    p->sz_values = bitmap_words_bytes(len);
  } else {
    p->sz_values = (size_t)(len > 0 ? len : 1) * type_width(p->type);
  }
  return QE_OK;
}

void batch_release_host(ArrowArray* a);
void schema_release(ArrowSchema* s);

struct HostExport {  // private_data of an exported ArrowArray
  std::vector<void*> blocks;
  std::vector<ArrowArray*> children;
  std::vector<const void*> bufs;  // 3 per child
};

void batch_release_host(ArrowArray* a) {
  if (!a || !a->release) return;
  HostExport* h = (HostExport*)a->private_data;
  for (ArrowArray* c : h->children) {
    free(c);
  }
  for (void* b : h->blocks) free(b);
  delete h;
  a->release = nullptr;
}

void child_release_noop(ArrowArray* a) { a->release = nullptr; }

struct SchemaPriv {
  std::vector<ArrowSchema*> children;
  std::vector<std::string> names;
};

void child_schema_release(ArrowSchema* s) { s->release = nullptr; }

void schema_release(ArrowSchema* s) {
  if (!s || !s->release) return;
  SchemaPriv* p = (SchemaPriv*)s->private_data;
  for (ArrowSchema* c : p->children) free(c);
  delete p;
  s->release = nullptr;
}

}  // namespace

int parallel_h2d_copy(qe_ctx* ctx, void* dst, const void* src, size_t n) {
  return parallel_h2d(ctx, std::vector<H2DJob>{{(uint8_t*)dst, (const uint8_t*)src, n}});
}

int parallel_h2d_file(qe_ctx* ctx, void* dst, int fd, int64_t off, size_t n) {
  return parallel_h2d(ctx, std::vector<H2DJob>{{(uint8_t*)dst, nullptr, n, fd, off}});
}

}  // namespace qe

using namespace qe;

extern "C" {

int qe_file_to_device(qe_ctx* ctx, const char* path, int64_t offset, int64_t bytes, void* dst) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(path && offset >= 0 && bytes >= 0 && (dst || bytes == 0), QE_ERR_INVALID_ARG, "bad arguments");
  if (bytes == 0) return QE_OK;
  const int fd = open(path, O_RDONLY | O_CLOEXEC);
  QE_CHECK(fd >= 0, QE_ERR_INVALID_ARG, "cannot open %s: %s", path, strerror(errno));
  (void)posix_fadvise(fd, offset, bytes, POSIX_FADV_SEQUENTIAL);
  const int rc = parallel_h2d_file(ctx, dst, fd, offset, (size_t)bytes);
  close(fd);
  return rc;
}

int qe_batch_import(qe_ctx* ctx, const ArrowSchema* schema, const ArrowArray* array, qe_batch** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(schema && array && out, QE_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  QE_CHECK(array->release != nullptr, QE_ERR_INVALID_ARG, "Arrow array already released");
  QE_CHECK(schema->format && !strcmp(schema->format, "+s"), QE_ERR_INVALID_ARG,
           "expected a struct array (record batch), got format '%s'", schema->format ? schema->format : "?");
  QE_CHECK(schema->n_children == array->n_children, QE_ERR_INVALID_ARG, "schema/array child count mismatch");
  const int64_t n = array->length;
  const int64_t nc = array->n_children;
  std::vector<ColPlan> plans((size_t)nc);
  size_t total = 0;
  for (int64_t i = 0; i < nc; ++i) {
    ColPlan& p = plans[(size_t)i];
    QE_TRY(plan_column(schema->children[i], array->children[i], array->offset, n, &p));
    p.o_valid = total;
    total += align256(p.sz_valid);
    p.o_offs = total;
    total += align256(p.sz_offs);
    p.o_values = total;
    total += align256(p.sz_values);
  }
  qe_batch* b = new qe_batch();
  b->ctx = ctx;
  b->length = n;
  if (dev_alloc(ctx, total ? total : 256, &b->device_block) != QE_OK) {
    delete b;
    return fail(QE_ERR_OOM, "device allocation of %zu bytes for an imported batch failed", total);
  }
  uint8_t* base = (uint8_t*)b->device_block;
  std::vector<H2DJob> jobs;
  std::vector<std::vector<uint8_t>> keep;  // rebased / realigned host buffers, alive until the copy
  for (int64_t i = 0; i < nc; ++i) {
    const ColPlan& p = plans[(size_t)i];
    qe_column c{};
    c.type = p.type;
    c.length = n;
    if (p.validity) {
      keep.emplace_back(p.sz_valid);
      copy_bits(keep.back().data(), p.validity, p.off, n, p.sz_valid);
      jobs.push_back({base + p.o_valid, keep.back().data(), p.sz_valid});
      c.validity = base + p.o_valid;
    }
    c.values = base + p.o_values;
    if (p.type == QE_TYPE_UTF8) {
      keep.emplace_back(p.sz_offs);
      int32_t* offs = (int32_t*)keep.back().data();
      for (int64_t r = 0; r <= n; ++r)
        offs[r] = p.large ? (int32_t)(((const int64_t*)p.offsets)[p.off + r] - p.byte0)
                          : (int32_t)(((const int32_t*)p.offsets)[p.off + r] - p.byte0);
      jobs.push_back({base + p.o_offs, keep.back().data(), p.sz_offs});
      if (p.nbytes > 0) jobs.push_back({(uint8_t*)c.values, (const uint8_t*)p.values + p.byte0, (size_t)p.nbytes});
      c.offsets = (int32_t*)(base + p.o_offs);
    } else if (p.type == QE_TYPE_BOOL) {
      keep.emplace_back(p.sz_values);
      copy_bits(keep.back().data(), (const uint8_t*)p.values, p.off, n, p.sz_values);
      jobs.push_back({(uint8_t*)c.values, keep.back().data(), p.sz_values});
    } else if (n > 0) {
      const int w = type_width(p.type);
      jobs.push_back({(uint8_t*)c.values, (const uint8_t*)p.values + p.off * w, (size_t)n * w});
    }
    b->cols.push_back(c);
    b->names.push_back(schema->children[i]->name ? schema->children[i]->name : "");
  }
  const int rc = parallel_h2d(ctx, jobs);
  if (rc != QE_OK) {
    dev_free(ctx, b->device_block);
    delete b;
    return rc;
  }
  *out = b;
  return QE_OK;
}

int qe_batch_import_device(qe_ctx* ctx, const ArrowSchema* schema, const ArrowDeviceArray* darray, qe_batch** out) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(schema && darray && out, QE_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  QE_CHECK(darray->device_type == QE_ARROW_DEVICE_ROCM && darray->device_id == ctx->device, QE_ERR_INVALID_ARG,
           "device array is on device type %d id %lld, context is ROCm device %d", darray->device_type,
           (long long)darray->device_id, ctx->device);
  if (darray->sync_event) QE_HIP(hipStreamWaitEvent(ctx->stream, *(hipEvent_t*)darray->sync_event, 0));
  const ArrowArray* array = &darray->array;
  QE_CHECK(schema->format && !strcmp(schema->format, "+s"), QE_ERR_INVALID_ARG, "expected a struct array");
  QE_CHECK(schema->n_children == array->n_children, QE_ERR_INVALID_ARG, "schema/array child count mismatch");
  qe_batch* b = new qe_batch();
  b->ctx = ctx;
  b->length = array->length;
  for (int64_t i = 0; i < array->n_children; ++i) {
    const ArrowSchema* s = schema->children[i];
    const ArrowArray* a = array->children[i];
    qe_column c{};
    c.type = type_of_format(s->format);
    const int64_t off = a->offset + array->offset;
    const bool ok = c.type != 0 && c.type != QE_TYPE_BOOL && strcmp(s->format, "U") != 0 &&
                    (a->null_count == 0 || a->buffers[0] == nullptr || (off & 31) == 0);
    if (!ok) {
      delete b;
      return fail(QE_ERR_UNSUPPORTED,
                  "zero-copy import of field %s (format '%s', offset %lld) is not supported; use qe_batch_import",
                  s->name ? s->name : "?", s->format ? s->format : "?", (long long)off);
    }
    c.length = array->length;
    if (a->null_count != 0 && a->buffers[0]) c.validity = (uint8_t*)a->buffers[0] + off / 8;
    if (c.type == QE_TYPE_UTF8) {
      c.offsets = (int32_t*)a->buffers[1] + off;  // byte positions stay absolute into buffers[2]
      c.values = (void*)a->buffers[2];
    } else {
      c.values = (uint8_t*)a->buffers[1] + off * type_width(c.type);
    }
    b->cols.push_back(c);
    b->names.push_back(s->name ? s->name : "");
  }
  *out = b;
  return QE_OK;
}

int qe_batch_destroy(qe_batch* b) {
  if (!b) return QE_OK;
  if (b->device_block) {
    (void)hipSetDevice(b->ctx->device);
    dev_free(b->ctx, b->device_block);
  }
  delete b;
  return QE_OK;
}

int qe_batch_num_columns(const qe_batch* b, int32_t* ncols, int64_t* length) {
  QE_CHECK(b, QE_ERR_INVALID_ARG, "null batch");
  if (ncols) *ncols = (int32_t)b->cols.size();
  if (length) *length = b->length;
  return QE_OK;
}

int qe_batch_column(const qe_batch* b, int32_t i, qe_column* out, const char** name) {
  QE_CHECK(b && out, QE_ERR_INVALID_ARG, "null argument");
  QE_CHECK(i >= 0 && (size_t)i < b->cols.size(), QE_ERR_INVALID_ARG, "column %d out of range", i);
  *out = b->cols[(size_t)i];
  if (name) *name = b->names[(size_t)i].c_str();
  return QE_OK;
}

int qe_batch_export(qe_ctx* ctx, const qe_column* cols, int32_t ncols, const char* const* names,
                    ArrowSchema* out_schema, ArrowArray* out_array) {
  QE_TRY(ctx_enter(ctx));
  QE_CHECK(out_schema && out_array && (cols || ncols == 0), QE_ERR_INVALID_ARG, "null argument");
  const int64_t n = ncols > 0 ? cols[0].length : 0;
  for (int32_t i = 0; i < ncols; ++i) {
    QE_CHECK(cols[i].length == n, QE_ERR_INVALID_ARG, "column %d has %lld rows, expected %lld", i,
             (long long)cols[i].length, (long long)n);
    QE_CHECK(format_of_type(cols[i].type) != nullptr, QE_ERR_UNSUPPORTED, "cannot export type %d", cols[i].type);
  }
  HostExport* h = new HostExport();
  h->bufs.resize((size_t)ncols * 3 + 1, nullptr);
  // children arrays: one malloc each (ArrowArray + 3 buffer pointers live in h->bufs)
  int rc = QE_OK;
  for (int32_t i = 0; i < ncols && rc == QE_OK; ++i) {
    const qe_column& c = cols[i];
    ArrowArray* a = (ArrowArray*)calloc(1, sizeof(ArrowArray));
    h->children.push_back(a);
    const void** bufs = &h->bufs[(size_t)i * 3];
    int64_t nulls = 0;
    if (c.validity) {
      const size_t vb = (size_t)div_up((uint64_t)(n > 0 ? n : 1), 8);
      uint8_t* v = (uint8_t*)malloc(vb + 8);
      h->blocks.push_back(v);
      if (hipMemcpyAsync(v, c.validity, vb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = QE_ERR_DEVICE;
      bufs[0] = v;
    }
    if (c.type == QE_TYPE_UTF8) {
      int32_t* o = (int32_t*)malloc((size_t)(n + 1) * 4);
      h->blocks.push_back(o);
      if (hipMemcpyAsync(o, c.offsets, (size_t)(n + 1) * 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
          hipStreamSynchronize(ctx->stream) != hipSuccess)
        rc = QE_ERR_DEVICE;
      const int32_t o0 = rc == QE_OK ? o[0] : 0;
      const int64_t nb = rc == QE_OK ? (int64_t)o[n] - o0 : 0;
      for (int64_t r = 0; rc == QE_OK && r <= n; ++r) o[r] -= o0;
      uint8_t* d = (uint8_t*)malloc((size_t)(nb > 0 ? nb : 1));
      h->blocks.push_back(d);
      if (rc == QE_OK && nb > 0 &&
          hipMemcpyAsync(d, (const uint8_t*)c.values + o0, (size_t)nb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
        rc = QE_ERR_DEVICE;
      bufs[1] = o;
      bufs[2] = d;
      a->n_buffers = 3;
    } else {
      const size_t vb = c.type == QE_TYPE_BOOL ? (size_t)div_up((uint64_t)(n > 0 ? n : 1), 8)
                                               : (size_t)(n > 0 ? n : 1) * type_width(c.type);
      uint8_t* v = (uint8_t*)malloc(vb + 8);
      h->blocks.push_back(v);
      if (n > 0 && hipMemcpyAsync(v, c.values, vb, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess) rc = QE_ERR_DEVICE;
      bufs[1] = v;
      a->n_buffers = 2;
    }
    if (rc == QE_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) rc = QE_ERR_DEVICE;
    if (rc == QE_OK && c.validity) {
      const uint8_t* v = (const uint8_t*)bufs[0];
      int64_t valid = 0;
      for (int64_t r = 0; r < n / 8; ++r) valid += __builtin_popcount(v[r]);
      for (int64_t r = n & ~7ll; r < n; ++r) valid += (v[r >> 3] >> (r & 7)) & 1;
      nulls = n - valid;
    }
    a->length = n;
    a->null_count = nulls;
    a->offset = 0;
    a->n_children = 0;
    a->buffers = bufs;
    a->release = child_release_noop;
  }
  if (rc != QE_OK) {
    for (ArrowArray* c : h->children) free(c);
    for (void* p : h->blocks) free(p);
    delete h;
    return fail(QE_ERR_DEVICE, "device-to-host copy failed while exporting a batch");
  }
  memset(out_array, 0, sizeof(*out_array));
  out_array->length = n;
  out_array->null_count = 0;
  out_array->n_buffers = 1;
  out_array->buffers = &h->bufs[(size_t)ncols * 3];  // struct validity: none
  out_array->n_children = ncols;
  out_array->children = h->children.data();
  out_array->release = batch_release_host;
  out_array->private_data = h;

  SchemaPriv* sp = new SchemaPriv();
  for (int32_t i = 0; i < ncols; ++i) {
    ArrowSchema* s = (ArrowSchema*)calloc(1, sizeof(ArrowSchema));
    sp->names.push_back(names && names[i] ? names[i] : ("f" + std::to_string(i)));
    sp->children.push_back(s);
  }
  for (int32_t i = 0; i < ncols; ++i) {
    ArrowSchema* s = sp->children[(size_t)i];
    s->format = format_of_type(cols[i].type);
    s->name = sp->names[(size_t)i].c_str();
    s->flags = 2;  // ARROW_FLAG_NULLABLE: every field is nullable (K:31)
    s->release = child_schema_release;
  }
  memset(out_schema, 0, sizeof(*out_schema));
  out_schema->format = "+s";
  out_schema->name = "";
  out_schema->n_children = ncols;
  out_schema->children = sp->children.data();
  out_schema->release = schema_release;
  out_schema->private_data = sp;
  return QE_OK;
}

}  // extern "C"
