// Data-parallel gradient exchange over RCCL (xGMI) behind the C ABI: md2_comm_* and the
// overlapped bucket all-reduce of the model's backward (the reference
// loop that would call it is scripts/script.jl:84-86, gradient(θ) + update!).
//
// RCCL is bound at run time (dlopen of librccl.so.1, RTLD_LOCAL): the library has no link-time
// dependency on it, and in a process that already loaded RCCL (PyTorch) the loaded copy is
// reused.  MD2_RCCL_LIB names another library exporting the same five nccl* symbols (the tests'
// call-recording stub); it is tried first.  One communicator = one rank on one device + its own non-blocking comm stream.  The
// backward runs on the caller's stream; after segment k is enqueued an event orders the RCCL sum
// of that segment's (now final) gradient range on the comm stream, so the all-reduce of the
// decoder / deep encoder stages overlaps the remaining backward; the caller's stream then waits
// for every bucket before ADAM applies 1/nranks.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <rccl/rccl.h>

#include "model.h"

namespace md2 {
namespace {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  // optional (the tests' recording stub exports only the five above): the communicator's own
  // view of its size and rank, reported by md2_comm_rank
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*user_rank)(const ncclComm_t, int*) = nullptr;
};

int rccl(Rccl** out) {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    // MD2_RCCL_LIB swaps in the tests' call-recording stand-in (tests/stubs/rccl_stub.cpp).  A
    // production run that inherited it would silently not reduce across ranks, so it is honoured
    // only together with MD2_TUNING=1 (the test-and-tuning gate) and announced on stderr.
    const char* over = std::getenv("MD2_RCCL_LIB");
    const char* tun = std::getenv("MD2_TUNING");
    if (over && *over) {
      if (tun && std::strcmp(tun, "1") == 0) {
        std::fprintf(stderr, "libmd2hip: MD2_RCCL_LIB=%s replaces librccl (test stand-in)\n", over);
      } else {
        std::fprintf(stderr, "libmd2hip: ignoring MD2_RCCL_LIB=%s (needs MD2_TUNING=1)\n", over);
        over = nullptr;
      }
    }
    const char* names[] = {over, "librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if (n && *n && (r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
    if (r.h) {
      r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
      r.init_rank = (decltype(r.init_rank))dlsym(r.h, "ncclCommInitRank");
      r.destroy = (decltype(r.destroy))dlsym(r.h, "ncclCommDestroy");
      r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
      r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
      r.comm_count = (decltype(r.comm_count))dlsym(r.h, "ncclCommCount");
      r.user_rank = (decltype(r.user_rank))dlsym(r.h, "ncclCommUserRank");
    }
  }
  if (!r.h || !r.get_unique_id || !r.init_rank || !r.destroy || !r.all_reduce || !r.error_string) {
    set_error("RCCL (librccl.so.1) could not be loaded");
    return MD2_ENOTSUP;
  }
  *out = &r;
  return MD2_OK;
}

#define MD2_RCCL(R, expr)                                                                  \
  do {                                                                                     \
    ncclResult_t _r = (expr);                                                              \
    if (_r != ncclSuccess) {                                                               \
      ::md2::set_error(std::string("RCCL error ") + (R)->error_string(_r) + " (" #expr ")"); \
      return MD2_EHIP;                                                                     \
    }                                                                                      \
  } while (0)

}  // namespace
}  // namespace md2

using namespace md2;

struct md2_comm {
  Rccl* r = nullptr;
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1, device = 0;
  hipStream_t stream = nullptr;              // RCCL's stream (the buckets)
  std::vector<hipEvent_t> ready;             // per bucket: its gradient range is final
  hipEvent_t done = nullptr;                 // every bucket reduced
  long long calls = 0, bytes = 0;            // all-reduces enqueued and their payload (md2_comm_stats)
};

namespace {
// every all-reduce of the library goes through here (counted for md2_comm_stats)
ncclResult_t comm_allreduce(md2_comm* c, float* buf, size_t n, hipStream_t st) {
  ++c->calls;
  c->bytes += (long long)n * (long long)sizeof(float);
  return c->r->all_reduce(buf, buf, n, ncclFloat32, ncclSum, c->comm, st);
}
}  // namespace

extern "C" {

int md2_comm_get_unique_id(char* id) {
  MD2_CHECK_ARG(id, "id");
  Rccl* r;
  MD2_TRY(rccl(&r));
  ncclUniqueId u;
  MD2_RCCL(r, r->get_unique_id(&u));
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return MD2_OK;
}

int md2_comm_init(int rank, int nranks, const char* id, int device, md2_comm** out) {
  MD2_CHECK_ARG(out && id && nranks >= 1 && rank >= 0 && rank < nranks && device >= 0, "comm_init args");
  Rccl* r;
  MD2_TRY(rccl(&r));
  // RCCL binds the communicator and the comm stream to the CURRENT device: switch to `device`
  // for the setup and give the caller its own current device back on every path
  int prev = 0;
  MD2_HIP(hipGetDevice(&prev));
  MD2_HIP(hipSetDevice(device));
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  md2_comm* c = new md2_comm();
  c->r = r;
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  ncclUniqueId u;
  std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t rc = r->init_rank(&c->comm, nranks, u, rank);
  if (rc != ncclSuccess) {
    set_error(std::string("ncclCommInitRank: ") + r->error_string(rc));
    delete c;
    return MD2_EHIP;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
    set_error("comm stream / event creation failed");
    r->destroy(c->comm);
    delete c;
    return MD2_EHIP;
  }
  *out = c;
  return MD2_OK;
}

int md2_comm_destroy(md2_comm* c) {
  if (!c) return MD2_OK;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) c->r->destroy(c->comm);
  for (hipEvent_t e : c->ready) (void)hipEventDestroy(e);
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return MD2_OK;
}

int md2_comm_rank(const md2_comm* c, int* rank, int* nranks) {
  MD2_CHECK_ARG(c, "comm");
  int r = c->rank, n = c->nranks;
  // RCCL's own answer where the loaded library exports it (what the bench reports as the
  // communicator's size); the values given to md2_comm_init otherwise
  if (c->r->user_rank) MD2_RCCL(c->r, c->r->user_rank(c->comm, &r));
  if (c->r->comm_count) MD2_RCCL(c->r, c->r->comm_count(c->comm, &n));
  if (rank) *rank = r;
  if (nranks) *nranks = n;
  return MD2_OK;
}

int md2_comm_stats(const md2_comm* c, long long* calls, long long* bytes) {
  MD2_CHECK_ARG(c, "comm");
  if (calls) *calls = c->calls;
  if (bytes) *bytes = c->bytes;
  return MD2_OK;
}

int md2_comm_allreduce_sum(md2_comm* c, float* buf, long long n, void* stream) {
  MD2_CHECK_ARG(c && buf && n >= 0, "allreduce args");
  MD2_RCCL(c->r, comm_allreduce(c, buf, (size_t)n, (hipStream_t)stream));
  return MD2_OK;
}

int md2_model_backward_allreduce(md2_model* m, md2_comm* c, void* stream) {
  MD2_CHECK_ARG(m, "model");
  hipStream_t st = (hipStream_t)stream;
  const int nseg = model_num_segments(m->impl);
  if (!c) {
    for (int k = 0; k < nseg; ++k) MD2_TRY(model_backward_segment(m->impl, k, nullptr, nullptr, st));
    return MD2_OK;
  }
  while ((int)c->ready.size() < nseg) {
    hipEvent_t e;
    MD2_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ready.push_back(e);
  }
  float* g = model_grads(m->impl);
  for (int k = 0; k < nseg; ++k) {
    long off = 0, len = 0;
    MD2_TRY(model_backward_segment(m->impl, k, &off, &len, st));
    MD2_HIP(hipEventRecord(c->ready[k], st));
    MD2_HIP(hipStreamWaitEvent(c->stream, c->ready[k], 0));
    MD2_RCCL(c->r, comm_allreduce(c, g + off, (size_t)len, c->stream));
  }
  MD2_HIP(hipEventRecord(c->done, c->stream));
  MD2_HIP(hipStreamWaitEvent(st, c->done, 0));
  return MD2_OK;
}

int md2_model_train_step_dp(md2_model* m, md2_comm* c, const float* x, const float* auto_loss,
                            float* adam_m, float* adam_v, float lr, float beta1, float beta2,
                            float eps, int step, float* loss, void* stream) {
  MD2_CHECK_ARG(m && x && adam_m && adam_v && step >= 1, "train_step_dp args");
  hipStream_t st = (hipStream_t)stream;
  MD2_TRY(model_forward_loss(m->impl, x, auto_loss, loss, nullptr, st));
  const float scale = c ? 1.f / (float)c->nranks : 1.f;
  if (!model_segment_update_enabled()) {   // measured default: one update after the last bucket
    MD2_TRY(md2_model_backward_allreduce(m, c, stream));
    return model_adam(m->impl, adam_m, adam_v, lr, beta1, beta2, eps, step, scale, st);
  }
  const int nseg = model_num_segments(m->impl);
  if (!c) {
    for (int k = 0; k < nseg; ++k) {
      MD2_TRY(model_backward_segment(m->impl, k, nullptr, nullptr, st));
      MD2_TRY(model_adam_segment(m->impl, k, adam_m, adam_v, lr, beta1, beta2, eps, step, scale, st));
    }
    return model_adam_join(m->impl, st);
  }
  while ((int)c->ready.size() < nseg) {
    hipEvent_t e;
    MD2_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ready.push_back(e);
  }
  // per bucket: the segment's backward on st, its all-reduce on the comm stream, then its ADAM +
  // re-pack on the executor's update stream ordered after that all-reduce (model_adam_segment)
  float* g = model_grads(m->impl);
  for (int k = 0; k < nseg; ++k) {
    long off = 0, len = 0;
    MD2_TRY(model_backward_segment(m->impl, k, &off, &len, st));
    MD2_HIP(hipEventRecord(c->ready[k], st));
    MD2_HIP(hipStreamWaitEvent(c->stream, c->ready[k], 0));
    MD2_RCCL(c->r, comm_allreduce(c, g + off, (size_t)len, c->stream));
    MD2_TRY(model_adam_segment(m->impl, k, adam_m, adam_v, lr, beta1, beta2, eps, step, scale, c->stream));
  }
  MD2_HIP(hipEventRecord(c->done, c->stream));
  MD2_HIP(hipStreamWaitEvent(st, c->done, 0));
  return model_adam_join(m->impl, st);
}

}  // extern "C"
