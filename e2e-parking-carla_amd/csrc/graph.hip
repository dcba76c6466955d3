// HIP-graph surgery for captured train steps.
//
// On this ROCm stack a memset node captured into a HIP graph (hipMemsetAsync / D8 / D32
// during stream capture) replays correctly only on the first launch of the instantiated
// graph; later launches leave garbage (scripts/diag_memset3.py shows it in isolation).
// PyTorch's reductions zero their cross-block semaphores with hipMemsetAsync, so a captured
// backward silently corrupts bias gradients from the second replay on.  Before
// instantiation, every memset node is replaced here by an equivalent kernel node (same
// dependencies, same dependents) running k_memset_node; memcpy and kernel nodes are left
// alone.
#include <unordered_set>
#include <vector>

#include "common.h"

namespace e2ep {

__global__ void k_memset_node(char *dst, size_t pitch, size_t width, size_t height,
                              unsigned value, int esz) {
  const size_t total = width * height;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / width, c = i - r * width;
    char *p = dst + r * pitch + c * esz;
    if (esz == 4)
      *reinterpret_cast<unsigned *>(p) = value;
    else if (esz == 2)
      *reinterpret_cast<unsigned short *>(p) = (unsigned short)value;
    else
      *p = (char)value;
  }
}

}  // namespace e2ep

using namespace e2ep;

#define E2EP_HIPCHECK(call)                                          \
  do {                                                               \
    hipError_t e_ = (call);                                          \
    if (e_ != hipSuccess) {                                          \
      set_error("%s: %s", #call, hipGetErrorString(e_));             \
      return (int)e_;                                                \
    }                                                                \
  } while (0)

extern "C" {

int e2ep_graph_replace_memsets(void *graph, int *replaced) {
  E2EP_REQUIRE(graph != nullptr, E2EP_EINVAL, "e2ep_graph_replace_memsets: null graph");
  hipGraph_t g = static_cast<hipGraph_t>(graph);
  size_t n = 0;
  E2EP_HIPCHECK(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) E2EP_HIPCHECK(hipGraphGetNodes(g, nodes.data(), &n));
  int count = 0;
  for (size_t k = 0; k < n; ++k) {
    hipGraphNodeType t;
    E2EP_HIPCHECK(hipGraphNodeGetType(nodes[k], &t));
    if (t != hipGraphNodeTypeMemset) continue;
    hipMemsetParams mp;
    E2EP_HIPCHECK(hipGraphMemsetNodeGetParams(nodes[k], &mp));
    size_t nd = 0, nn = 0;
    E2EP_HIPCHECK(hipGraphNodeGetDependencies(nodes[k], nullptr, &nd));
    E2EP_HIPCHECK(hipGraphNodeGetDependentNodes(nodes[k], nullptr, &nn));
    std::vector<hipGraphNode_t> deps(nd), dents(nn);
    if (nd) E2EP_HIPCHECK(hipGraphNodeGetDependencies(nodes[k], deps.data(), &nd));
    if (nn) E2EP_HIPCHECK(hipGraphNodeGetDependentNodes(nodes[k], dents.data(), &nn));

    char *dst = static_cast<char *>(mp.dst);
    size_t pitch = mp.pitch, width = mp.width, height = mp.height ? mp.height : 1;
    unsigned value = mp.value;
    int esz = (int)mp.elementSize;
    E2EP_REQUIRE(esz == 1 || esz == 2 || esz == 4, E2EP_ERANGE,
                 "e2ep_graph_replace_memsets: element size %d", esz);
    void *args[] = {&dst, &pitch, &width, &height, &value, &esz};
    const size_t total = width * height;
    hipKernelNodeParams kp = {};
    kp.func = reinterpret_cast<void *>(k_memset_node);
    kp.blockDim = dim3(256);
    kp.gridDim = dim3((unsigned)(total / 256 + 1 < 1024 ? total / 256 + 1 : 1024));
    kp.sharedMemBytes = 0;
    kp.kernelParams = args;
    kp.extra = nullptr;
    hipGraphNode_t kn;
    E2EP_HIPCHECK(hipGraphAddKernelNode(&kn, g, nd ? deps.data() : nullptr, nd, &kp));
    for (size_t d = 0; d < nn; ++d) E2EP_HIPCHECK(hipGraphAddDependencies(g, &kn, &dents[d], 1));
    E2EP_HIPCHECK(hipGraphDestroyNode(nodes[k]));
    ++count;
  }
  if (replaced) *replaced = count;
  return 0;
}

// Own executable of a captured graph, launched without PyTorch's CUDAGraph.replay(): that
// replay's prologue refreshes the philox seed / offset tensors of torch's generators with
// int64 fill kernels (at::native FillFunctor<long>) before the launch; the train step draws
// its random numbers from e2ep_rng_draw, so those launches are pure overhead in the step.
int e2ep_graph_exec_create(void *graph, void **exec) {
  E2EP_REQUIRE(graph && exec, E2EP_EINVAL, "e2ep_graph_exec_create: null argument");
  hipGraphExec_t e = nullptr;
  E2EP_HIPCHECK(hipGraphInstantiate(&e, static_cast<hipGraph_t>(graph), nullptr, nullptr, 0));
  *exec = e;
  return 0;
}

int e2ep_graph_exec_launch(void *exec, void *stream) {
  E2EP_REQUIRE(exec, E2EP_EINVAL, "e2ep_graph_exec_launch: null exec");
  E2EP_HIPCHECK(hipGraphLaunch(static_cast<hipGraphExec_t>(exec), as_stream(stream)));
  return 0;
}

int e2ep_graph_exec_destroy(void *exec) {
  if (exec) E2EP_HIPCHECK(hipGraphExecDestroy(static_cast<hipGraphExec_t>(exec)));
  return 0;
}

// An unjoined side stream at hipStreamEndCapture: the round-2 / round-4 nested-fork captures
// segfaulted there instead of failing.  `side`'s capture frontier (the nodes its next work
// would depend on) must lie among the ancestors of `origin`'s frontier.
int e2ep_capture_unjoined(void *origin, void *side, int *unjoined) {
  E2EP_REQUIRE(unjoined, E2EP_EINVAL, "e2ep_capture_unjoined: null result");
  *unjoined = 0;
  hipStreamCaptureStatus so = hipStreamCaptureStatusNone, ss = hipStreamCaptureStatusNone;
  unsigned long long io = 0, is = 0;
  hipGraph_t go = nullptr, gs = nullptr;
  const hipGraphNode_t *d = nullptr;
  size_t n = 0;
  E2EP_HIPCHECK(hipStreamGetCaptureInfo_v2(as_stream(origin), &so, &io, &go, &d, &n));
  E2EP_REQUIRE(so == hipStreamCaptureStatusActive, E2EP_EINVAL,
               "e2ep_capture_unjoined: the origin stream is not capturing");
  std::vector<hipGraphNode_t> frontier(d, d + n);
  d = nullptr;
  n = 0;
  E2EP_HIPCHECK(hipStreamGetCaptureInfo_v2(as_stream(side), &ss, &is, &gs, &d, &n));
  if (ss != hipStreamCaptureStatusActive || is != io || n == 0) return 0;
  std::vector<hipGraphNode_t> tail(d, d + n);
  std::unordered_set<hipGraphNode_t> seen(frontier.begin(), frontier.end());
  std::vector<hipGraphNode_t> stack(frontier);
  std::vector<hipGraphNode_t> deps;
  while (!stack.empty()) {
    hipGraphNode_t x = stack.back();
    stack.pop_back();
    size_t nd = 0;
    E2EP_HIPCHECK(hipGraphNodeGetDependencies(x, nullptr, &nd));
    deps.resize(nd);
    if (nd) E2EP_HIPCHECK(hipGraphNodeGetDependencies(x, deps.data(), &nd));
    for (size_t k = 0; k < nd; ++k)
      if (seen.insert(deps[k]).second) stack.push_back(deps[k]);
  }
  for (hipGraphNode_t t : tail)
    if (!seen.count(t)) *unjoined = 1;
  return 0;
}

}  // extern "C"
