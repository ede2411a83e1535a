// Native hipGraph capture / upload / launch for whole training steps.
//
// torch.cuda.CUDAGraph instantiates at capture end but does not stage the executable
// graph on the device; its first replay pays the upload (kernel-object descriptors and
// the AQL packet chain of every node) inside whatever region the caller is timing.
// The trainer's step launches only this library's kernels (ctypes, no torch ops, no
// allocations), so it can be captured directly with the HIP runtime:
//
//   pto_graph_begin(stream)         hipStreamBeginCapture (thread-local mode)
//   ... K whole training steps ...  (the launchers record onto `stream`)
//   pto_graph_end(stream, &h)       hipStreamEndCapture + hipGraphInstantiate
//   pto_graph_upload(h, stream)     hipGraphUpload: device-side staging, no execution
//   pto_graph_launch(h, stream, n)  n back-to-back hipGraphLaunch
//   pto_graph_destroy(h)
//
// `stream` must be a non-default stream (capture on the null stream is invalid).
#include <hip/hip_runtime.h>

#include <new>

namespace {
struct PtoGraph {
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  size_t nodes = 0;
};
}  // namespace

extern "C" {

int pto_graph_begin(void* stream) {
  if (stream == nullptr) return -1;
  return (int)hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal);
}

int pto_graph_end(void* stream, void** out) {
  if (stream == nullptr || out == nullptr) return -1;
  *out = nullptr;
  hipGraph_t g = nullptr;
  hipError_t e = hipStreamEndCapture((hipStream_t)stream, &g);
  if (e != hipSuccess) return (int)e;
  if (g == nullptr) return -1;
  PtoGraph* h = new (std::nothrow) PtoGraph();
  if (h == nullptr) {
    (void)hipGraphDestroy(g);
    return -1;
  }
  h->graph = g;
  (void)hipGraphGetNodes(g, nullptr, &h->nodes);
  e = hipGraphInstantiate(&h->exec, g, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    (void)hipGraphDestroy(g);
    delete h;
    return (int)e;
  }
  *out = h;
  return 0;
}

int pto_graph_upload(void* handle, void* stream) {
  auto* h = static_cast<PtoGraph*>(handle);
  if (h == nullptr || h->exec == nullptr) return -1;
  return (int)hipGraphUpload(h->exec, (hipStream_t)stream);
}

int pto_graph_launch(void* handle, void* stream, int n) {
  auto* h = static_cast<PtoGraph*>(handle);
  if (h == nullptr || h->exec == nullptr || n < 0) return -1;
  for (int i = 0; i < n; ++i) {
    const hipError_t e = hipGraphLaunch(h->exec, (hipStream_t)stream);
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

long pto_graph_nodes(void* handle) {
  auto* h = static_cast<PtoGraph*>(handle);
  return h == nullptr ? -1 : (long)h->nodes;
}

int pto_graph_destroy(void* handle) {
  auto* h = static_cast<PtoGraph*>(handle);
  if (h == nullptr) return 0;
  hipError_t e = hipSuccess;
  if (h->exec != nullptr) e = hipGraphExecDestroy(h->exec);
  if (h->graph != nullptr) (void)hipGraphDestroy(h->graph);
  delete h;
  return (int)e;
}

}  // extern "C"
