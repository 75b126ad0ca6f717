// Call-recording stand-in for RCCL (test infrastructure: tests/test_gpu_dp.py).  Loaded by
// libmd2hip.so through MD2_RCCL_LIB in place of librccl.so.1; exports the five nccl* symbols the
// library binds.  ncclAllReduce does not reduce: it records (recv, count, stream) and enqueues a
// device-to-device copy of the bucket ON THE STREAM IT WAS GIVEN, so the copy sees the bucket as
// it is when the collective would run in stream order -- the test compares these snapshots with
// the final gradient to prove each bucket's collective is ordered after its backward segment.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <vector>

namespace {
struct Rec {
  void* recv;
  size_t count;
  hipStream_t stream;
  float* snap;
};
std::vector<Rec> g_log;
}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  std::memset(id, 0, sizeof(*id));
  return ncclSuccess;
}
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int, ncclUniqueId, int) {
  *comm = reinterpret_cast<ncclComm_t>(0x1);
  return ncclSuccess;
}
ncclResult_t ncclCommDestroy(ncclComm_t) { return ncclSuccess; }
const char* ncclGetErrorString(ncclResult_t) { return "rccl stub"; }
ncclResult_t ncclAllReduce(const void*, void* recv, size_t count, ncclDataType_t, ncclRedOp_t,
                           ncclComm_t, hipStream_t stream) {
  float* snap = nullptr;
  if (hipMalloc(&snap, count * sizeof(float) + 4) != hipSuccess) return ncclSystemError;
  if (hipMemcpyAsync(snap, recv, count * sizeof(float), hipMemcpyDeviceToDevice, stream) != hipSuccess)
    return ncclSystemError;
  g_log.push_back({recv, count, stream, snap});
  return ncclSuccess;
}

int stub_count() { return (int)g_log.size(); }
int stub_get(int i, void** recv, size_t* count, void** stream, void** snap) {
  if (i < 0 || i >= (int)g_log.size()) return 1;
  *recv = g_log[i].recv;
  *count = g_log[i].count;
  *stream = (void*)g_log[i].stream;
  *snap = g_log[i].snap;
  return 0;
}
void stub_reset() {
  for (Rec& r : g_log) (void)hipFree(r.snap);
  g_log.clear();
}

}  // extern "C"
