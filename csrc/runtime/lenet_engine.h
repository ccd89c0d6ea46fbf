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
  bf16* act2 = nullptr;          // [act2_rows][F0P]
  int act2_rows = 0;
  bf16* act2T = nullptr;         // [F0P][MAX_TRAIN_BATCH]
  bf16* h1 = nullptr;            // [act2_rows][128]  relu(fc1)
  bf16* pool1 = nullptr;         // [MAX_TRAIN_BATCH][NP1]
  uint8_t* am1 = nullptr;        // [MAX_TRAIN_BATCH][NP1]
  uint8_t* am2 = nullptr;        // [MAX_TRAIN_BATCH][F0]
  float* dact2 = nullptr;        // [MAX_TRAIN_BATCH][F0]  d(pool2) from the FC head
  bf16* dZ1T = nullptr;          // [DZ1_LD][MAX_TRAIN_BATCH]
  float* conv_slab = nullptr;    // [MAX_TRAIN_BATCH][CS]
  float* fc1w_grad = nullptr;    // [F1W_N]
  float* fc_slab = nullptr;      // [MAX_FC_WG][FS]
  lenet::Stats* train_stats = nullptr;
  lenet::Stats* eval_stats = nullptr;
  int* round_ctr = nullptr;      // augmentation epoch counter (device)
  int* done_flags = nullptr;     // [MAX_TRAIN_BATCH] K12 hand-off flags (optional: enables fuse_head)
  int* step_gen = nullptr;       // step generation, bumped by K4 / K34
  int* bwd_flags = nullptr;      // [MAX_TRAIN_BATCH + N_DW1_WG] K34 producer flags (optional: enables fuse_sgd)
  int* bwd_gen = nullptr;        // K34's flag generation, bumped by K12
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

  // One SGD step (eager launches) on samples [start, start+nb).
  void step(hipStream_t st, int start, int nb, bool bump_round, bool reset_stats = false);
  // One local epoch over the schedule; graph replay when use_graph.
  void run_epoch(hipStream_t st, bool use_graph);
  // Forward + CE/accuracy over n samples of an image set (eval mode).  pk / params (optional): read the
  // model from these copies instead of the live buffers (an eval that overlaps the next round's training).
  void eval(hipStream_t st, const uint8_t* images, const int* labels, int n, const bf16* pk = nullptr,
            const float* params = nullptr);
  // Refresh the packed bf16 images from the fp32 master (after FedAvg/load).
  void pack(hipStream_t st);
  void set_sgd(SgdConfig sgd);
  // fc1 computed inside the FC-tail kernel (4 launches per step) instead of its own kernel (5)
  void set_fuse_fc1(bool on);
  bool fuse_fc1() const { return fuse_fc1_; }
  bool graph_ready() const { return exec_ != nullptr; }
  // conv stack + FC head in one launch (K12) instead of K1 then K2 (needs done_flags/step_gen)
  void set_fuse_head(bool on);
  bool fuse_head() const { return fuse_head_; }
  // conv backward + SGD in one launch (K34) instead of K3 then K4 (needs fuse_head, bwd_flags/bwd_gen)
  void set_fuse_sgd(bool on);
  bool fuse_sgd() const { return fuse_sgd_; }
  // per-sample step (KS1: one workgroup runs a sample's whole forward + backward) + GEMM/SGD (KS2):
  // 2 launches per step, no inter-workgroup hand-off; takes precedence over fuse_head / fuse_sgd
  void set_sample_path(bool on);
  bool sample_path() const { return sample_path_; }

 private:
  void enqueue_epoch(hipStream_t st);
  void drop_graph();

  LeNetBuffers b_;
  SgdConfig sgd_;
  uint32_t seed_;
  bool augment_;
  bool fuse_fc1_ = false;
  bool fuse_head_ = false;
  bool fuse_sgd_ = false;
  bool sample_path_ = false;
  std::vector<int> starts_, sizes_;
  hipStream_t cap_stream_ = nullptr;
  hipGraph_t graph_ = nullptr;
  hipGraphExec_t exec_ = nullptr;
};

void check_hip(hipError_t e, const char* what);

}  // namespace fedmi
