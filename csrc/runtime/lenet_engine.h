// fedmi — native local-epoch executor for the fused LeNet kernels.
//
// Replaces the reference's per-batch Python loop (src/main.py:128-165: a
// DataLoader over ALL batches, skipping the ones not owned by this rank, two
// device->host syncs per step) with a schedule of only this rank's batches,
// captured ONCE into a hipGraph and replayed per federated round.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <vector>
#include "../kernels/lenet_layout.h"

namespace fedmi {

typedef __bf16 bf16;

struct LeNetBuffers {
  const uint8_t* train_images = nullptr;  // [n_train][3072] uint8 CHW
  const int* train_labels = nullptr;
  int n_train = 0;
  float* params = nullptr;       // [P_TOTAL] fp32 master (state_dict order)
  float* mom = nullptr;          // [P_TOTAL] momentum buffers
  bf16* pk = nullptr;            // [PK_TOTAL] packed bf16 operand images
  bf16* act2 = nullptr;          // [act2_rows][F0P]  eval activations (pool2 output)
  int act2_rows = 0;
  bf16* act2T = nullptr;         // [F0P][MAX_TRAIN_BATCH]  KS1 -> KS2 fc1 wgrad operand
  bf16* h1 = nullptr;            // [128][128]  KS1 -> KS2 relu(fc1), sample-contiguous rows (h1T)
  float* dact2 = nullptr;        // [MAX_TRAIN_BATCH][F0]  KS1's FC side buffers (AUX_*)
  bf16* dZ1T = nullptr;          // [DZ1_LD][MAX_TRAIN_BATCH]
  float* conv_slab = nullptr;    // [MAX_TRAIN_BATCH][CS]  per-sample conv gradients
  float* eval_part = nullptr;    // eval (loss, correct) partials per 16-row group
  long eval_part_floats = 0;
  lenet::Stats* train_stats = nullptr;
  lenet::Stats* eval_stats = nullptr;
  int* round_ctr = nullptr;      // augmentation epoch counter (device)
};

struct SgdConfig {
  float lr = 0.1f, momentum = 0.9f, weight_decay = 5e-4f;
};

class LeNetEngine {
 public:
  LeNetEngine(const LeNetBuffers& b, SgdConfig sgd, uint32_t seed, bool augment);
  ~LeNetEngine();
  LeNetEngine(const LeNetEngine&) = delete;
  LeNetEngine& operator=(const LeNetEngine&) = delete;

  // The batches this rank trains in one local epoch: (first sample, count).
  void set_schedule(const std::vector<int>& starts, const std::vector<int>& sizes);
  int schedule_len() const { return (int)starts_.size(); }

  // One SGD step (eager launches: KS1 lenet_sample_step + KS2 lenet_sgd2) on samples [start, start+nb).
  void step(hipStream_t st, int start, int nb, bool bump_round, bool reset_stats = false);
  // One local epoch over the schedule; graph replay when use_graph.
  void run_epoch(hipStream_t st, bool use_graph);
  // Forward + CE/accuracy over n samples of an image set (eval mode).
  void eval(hipStream_t st, const uint8_t* images, const int* labels, int n);
  // Refresh the packed bf16 images from the fp32 master (after FedAvg/load).
  void pack(hipStream_t st);
  void set_sgd(SgdConfig sgd);
  bool graph_ready() const { return exec_ != nullptr; }

 private:
  void enqueue_epoch(hipStream_t st);
  void drop_graph();

  LeNetBuffers b_;
  SgdConfig sgd_;
  uint32_t seed_;
  bool augment_;
  std::vector<int> starts_, sizes_;
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

void check_hip(hipError_t e, const char* what);

}  // namespace fedmi
