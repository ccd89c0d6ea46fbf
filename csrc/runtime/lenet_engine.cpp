// fedmi — native local-epoch executor (see lenet_engine.h).
#include "lenet_engine.h"

#include <stdexcept>
#include <string>

namespace fedmi {

using lenet::Stats;

// launchers (csrc/kernels/lenet_kernels.hip)
void launch_lenet_conv_fwd(hipStream_t, const uint8_t*, int, int, const bf16*, const float*, uint32_t,
                           const int*, int, bf16*, bf16*, int, bf16*, uint8_t*, uint8_t*, lenet::Stats*);
void launch_lenet_fc_eval(hipStream_t, const bf16*, const int*, int, const bf16*, const float*, float*, long,
                          lenet::Stats*);
void launch_lenet_pack(hipStream_t, const float*, bf16*);
void launch_lenet_zero_stats(hipStream_t, lenet::Stats*);
void launch_lenet_sample_step(hipStream_t, const uint8_t*, int, int, const bf16*, const float*, uint32_t, const int*,
                              int, const int*, bf16*, bf16*, float*, bf16*, float*);
void launch_lenet_sgd2(hipStream_t, float*, float*, bf16*, const float*, int, const bf16*, const bf16*, const float*,
                       const bf16*, float, float, float, int*, lenet::Stats*);

void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("fedmi HIP error in ") + what + ": " + hipGetErrorString(e));
}

LeNetEngine::LeNetEngine(const LeNetBuffers& b, SgdConfig sgd, uint32_t seed, bool augment)
    : b_(b), sgd_(sgd), seed_(seed), augment_(augment) {
  if (!b.params || !b.mom || !b.pk || !b.act2 || !b.act2T || !b.h1 || !b.dact2 || !b.dZ1T || !b.conv_slab ||
      !b.eval_part || !b.train_stats || !b.eval_stats || !b.round_ctr)
    throw std::invalid_argument("LeNetEngine: missing device buffer");
  if (b.act2_rows < lenet::MAX_TRAIN_BATCH) throw std::invalid_argument("LeNetEngine: act2_rows < 128");
  check_hip(hipStreamCreateWithFlags(&cap_stream_, hipStreamNonBlocking), "hipStreamCreate");
}

LeNetEngine::~LeNetEngine() {
  drop_graph();
  if (cap_stream_) (void)hipStreamDestroy(cap_stream_);
}

void LeNetEngine::drop_graph() {
  if (exec_) (void)hipGraphExecDestroy(exec_);
  if (graph_) (void)hipGraphDestroy(graph_);
  exec_ = nullptr;
  graph_ = nullptr;
}

void LeNetEngine::set_schedule(const std::vector<int>& starts, const std::vector<int>& sizes) {
  if (starts.size() != sizes.size()) throw std::invalid_argument("schedule: length mismatch");
  for (size_t i = 0; i < starts.size(); ++i) {
    if (sizes[i] <= 0 || sizes[i] > lenet::MAX_TRAIN_BATCH) throw std::invalid_argument("schedule: bad batch size");
    if (starts[i] < 0 || starts[i] + sizes[i] > b_.n_train) throw std::invalid_argument("schedule: batch out of range");
  }
  starts_ = starts;
  sizes_ = sizes;
  drop_graph();
}

void LeNetEngine::set_sgd(SgdConfig sgd) {
  sgd_ = sgd;
  drop_graph();
}

void LeNetEngine::step(hipStream_t st, int start, int nb, bool bump_round, bool reset_stats) {
  using namespace lenet;
  if (nb <= 0 || nb > MAX_TRAIN_BATCH || start < 0 || start + nb > b_.n_train)
    throw std::invalid_argument("LeNetEngine::step: batch out of range");
  const int aug = augment_ ? 1 : 0;
  if (reset_stats) launch_lenet_zero_stats(st, b_.train_stats);   // a kernel node, not a memset (graph replay)
  // the FC side buffers (h2T, dZ2T, dZ3T, bias grads, losses) live in the dact2 buffer, h1T in h1
  launch_lenet_sample_step(st, b_.train_images, start, nb, b_.pk, b_.params, seed_, b_.round_ctr, aug,
                           b_.train_labels + start, b_.act2T, b_.h1, b_.dact2, b_.dZ1T, b_.conv_slab);
  launch_lenet_sgd2(st, b_.params, b_.mom, b_.pk, b_.conv_slab, nb, b_.act2T, b_.h1, b_.dact2, b_.dZ1T, sgd_.lr,
                    sgd_.momentum, sgd_.weight_decay, bump_round ? b_.round_ctr : nullptr, b_.train_stats);
  check_hip(hipGetLastError(), "LeNetEngine::step launch");
}

void LeNetEngine::enqueue_epoch(hipStream_t st) {
  const size_t n = starts_.size();
  for (size_t i = 0; i < n; ++i) step(st, starts_[i], sizes_[i], i + 1 == n, i == 0);
}

void LeNetEngine::run_epoch(hipStream_t st, bool use_graph) {
  if (starts_.empty()) {   // rank owns no batch this round: keep the augmentation counter in step
    check_hip(hipMemsetAsync(b_.train_stats, 0, sizeof(Stats), st), "memset stats");
    return;
  }
  if (!use_graph) {
    enqueue_epoch(st);
    return;
  }
  if (!exec_) {
    check_hip(hipStreamBeginCapture(cap_stream_, hipStreamCaptureModeThreadLocal), "BeginCapture");
    try {
      enqueue_epoch(cap_stream_);
    } catch (...) {
      hipGraph_t g = nullptr;
      (void)hipStreamEndCapture(cap_stream_, &g);
      if (g) (void)hipGraphDestroy(g);
      throw;
    }
    check_hip(hipStreamEndCapture(cap_stream_, &graph_), "EndCapture");
    check_hip(hipGraphInstantiate(&exec_, graph_, nullptr, nullptr, 0), "GraphInstantiate");
  }
  check_hip(hipGraphLaunch(exec_, st), "GraphLaunch");
}

void LeNetEngine::eval(hipStream_t st, const uint8_t* images, const int* labels, int n) {
  using namespace lenet;
  if (n <= 0 || n > b_.act2_rows) throw std::invalid_argument("LeNetEngine::eval: n exceeds act2 capacity");
  launch_lenet_conv_fwd(st, images, 0, n, b_.pk, b_.params, seed_, b_.round_ctr, 0, b_.act2, nullptr, 0,
                        nullptr, nullptr, nullptr, b_.eval_stats);
  launch_lenet_fc_eval(st, b_.act2, labels, n, b_.pk, b_.params, b_.eval_part, b_.eval_part_floats, b_.eval_stats);
  check_hip(hipGetLastError(), "LeNetEngine::eval launch");
}

void LeNetEngine::pack(hipStream_t st) {
  launch_lenet_pack(st, b_.params, b_.pk);
  check_hip(hipGetLastError(), "LeNetEngine::pack launch");
}

}  // namespace fedmi
