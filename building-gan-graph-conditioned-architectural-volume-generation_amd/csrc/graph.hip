// One instantiated step graph re-used across batches (Trainer.step_fresh).
//
// A fresh batch records its critic iteration as a new graph (the same launch
// sequence as the previous batch's, other pointers and grid sizes).  Building
// an executable graph per batch and destroying the previous one costs ~3 ms
// of host time per step; updating ONE executable graph in place from the
// newly recorded graph (hipGraphExecUpdate) keeps its instantiation and skips
// the destroy.  These are host-side runtime calls, no kernels.
#include "common.h"

extern "C" int vg_graph_exec_update(void* exec, void* graph) {
  if (!exec || !graph) return VG_EINVAL;
  hipGraphNode_t err_node = nullptr;
  hipGraphExecUpdateResult result = hipGraphExecUpdateError;
  const hipError_t e = hipGraphExecUpdate(static_cast<hipGraphExec_t>(exec), static_cast<hipGraph_t>(graph),
                                          &err_node, &result);
  if (e == hipSuccess && result == hipGraphExecUpdateSuccess) return 0;
  (void)hipGetLastError();  // a refused update leaves no sticky error behind
  return VG_EGRAPH_TOPOLOGY;
}

extern "C" int vg_graph_launch(void* exec, void* stream) {
  if (!exec) return VG_EINVAL;
  return static_cast<int>(hipGraphLaunch(static_cast<hipGraphExec_t>(exec), static_cast<hipStream_t>(stream)));
}
