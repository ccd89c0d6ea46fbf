// fedmi — LeNet ("2-conv CNN") memory layout shared by the HIP kernels, the
// native epoch executor and (via the bindings) the Python side.
//
// Architecture parity: reference src/models/lenet.py:5-23
//   conv1 3->6 k5, relu, maxpool2, conv2 6->16 k5, relu, maxpool2,
//   fc1 400->120 relu, fc2 120->84 relu, fc3 84->10.
//
// Master weights: ONE flat fp32 buffer in state_dict order, so the FedAvg
// all-reduce and the checkpoint writer see the model as a single contiguous
// vector (reference averages key-by-key on the CPU: src/server.py:155-179).
#pragma once

namespace lenet {

// ---- geometry -------------------------------------------------------------
constexpr int IMG = 32, CIN = 3, C1 = 6, C2 = 16;
constexpr int O1 = 28, P1 = 14;          // conv1 out / pool1 out side
constexpr int O2 = 10, P2 = 5;           // conv2 out / pool2 out side
constexpr int NPOS1 = O1 * O1;           // 784
constexpr int NP1 = C1 * P1 * P1;        // 1176 pooled conv1 outputs
constexpr int NPOS2 = O2 * O2;           // 100
constexpr int F0 = C2 * P2 * P2;         // 400 flattened features
constexpr int F0P = 416;                 // act2 row stride (13 k-steps of 32)
constexpr int F1 = 120, F2 = 84, NCLS = 10;
constexpr int IMG_BYTES = CIN * IMG * IMG;  // 3072 (uint8 CHW, CIFAR format)

// MFMA reduction dims (K) of the channels-last implicit GEMMs.
//   conv1 fwd: k = g*8 + t, g = r*3 + s/2 (15 groups + 1 pad), t = (s&1)*4 + c (c<3)
//   conv2 fwd: k = (r*5+s)*8 + c (c<6), 25 groups -> 200, pad 224
//   conv2 dgrad: k = (r*5+s)*16 + o, 400, pad 416
constexpr int K1C = 128, K2C = 224, KDG = 400, KDGP = 416;

// ---- master parameters (fp32, state_dict order) ----------------------------
constexpr int P_C1W = 0;                 // conv1.weight [6,3,5,5]
constexpr int P_C1B = 450;               // conv1.bias   [6]
constexpr int P_C2W = 456;               // conv2.weight [16,6,5,5]
constexpr int P_C2B = 2856;              // conv2.bias   [16]
constexpr int P_F1W = 2872;              // fc1.weight   [120,400]
constexpr int P_F1B = 50872;             // fc1.bias     [120]
constexpr int P_F2W = 50992;             // fc2.weight   [84,120]
constexpr int P_F2B = 61072;             // fc2.bias     [84]
constexpr int P_F3W = 61156;             // fc3.weight   [10,84]
constexpr int P_F3B = 61996;             // fc3.bias     [10]
constexpr int P_TOTAL = 62006;

// Gradient staging (combined by KS2 at the next kernel boundary: deterministic, no global
// atomics): conv_slab [nb][CS] per-sample grads of params [0, P_F1W); the FC weight grads are
// KS2's batch GEMMs over KS1's sample-contiguous operands.
constexpr int CS = P_F1W;                // 2872
constexpr int FS = P_TOTAL - P_F1B;      // 11134
constexpr int F1W_N = P_F1B - P_F1W;     // 48000

// ---- packed bf16 operand images (written by the SGD/pack kernels) ----------
// Each image is laid out so a lane's 8 consecutive K elements of an MFMA
// operand fragment are one 16-byte load.  Padding is zero and never written.
constexpr int PK_W1C  = 0;                      // [16 o][128 k]       conv1 B
constexpr int PK_W2C  = PK_W1C + 16 * K1C;      // [16 o][224 k]       conv2 B
constexpr int PK_W2DG = PK_W2C + 16 * K2C;      // [16 c][416 (r,s,o)] conv2 dgrad B
constexpr int PK_FC1  = PK_W2DG + 16 * KDGP;    // [128 n][416 f]      fc1 fwd B
constexpr int PK_FC2  = PK_FC1 + 128 * F0P;     // [96 n][128 f]       fc2 fwd B (fc1's dX reuses PK_FC1)
constexpr int PK_FC2T = PK_FC2 + 96 * 128;      // [128 f][96 n]       fc2 dgrad B
constexpr int PK_FC3  = PK_FC2T + 128 * 96;     // [16 n][96 f]        fc3 fwd + dgrad (KS1 stages it in LDS)
constexpr int PK_TOTAL = PK_FC3 + 16 * 96;

// ---- training-step geometry -------------------------------------------------
constexpr int MAX_TRAIN_BATCH = 128;     // reference batch (src/main.py:140)
constexpr int FC_SPW = 16;               // samples per eval FC-head workgroup (one MFMA row tile)
constexpr int DZ1_LD = 128;              // dZ1 [B][128] and dZ1T [128][B] (B = 128)

// Stats block: train row written by KS2 (per-sample losses summed in sample order), eval row by
// lenet_eval_stats (row-group partials in group order) -- single writers, no atomics.
struct Stats {
  float loss_sum;   // sum over samples of CE loss
  int correct;      // argmax == label
  int count;        // samples seen
  int pad;
};

}  // namespace lenet
