// fedmi — host-side sanitizer driver for the native LeNet runtime.
//
// Built by tools/asan/build.sh with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code only
// (-Xarch_host -fsanitize=...; the gfx950 device code is not instrumented -- GPU ASan is not available on
// this pool).  It drives csrc/runtime/lenet_engine.cpp exactly as the Python trainer does: every device
// buffer of LeNetBuffers allocated, synthetic uint8 images, schedules with full and partial batches,
// eager and graph-replayed epochs, graph re-capture on every path switch (sample / head / fused-SGD),
// eval and pack, error paths (bad schedules, missing buffers) -- and fails on any sanitizer report or
// non-finite parameter.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <vector>

#include "runtime/lenet_engine.h"

using namespace fedmi;
using namespace lenet;

namespace {

template <class T>
T* dalloc(size_t n) {
  void* p = nullptr;
  check_hip(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)), "hipMalloc");
  check_hip(hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(T)), "hipMemset");
  return static_cast<T*>(p);
}

int failures = 0;
void expect(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}

}  // namespace

int main() {
  const int n_train = 1024, n_test = 512, rows = std::max(MAX_TRAIN_BATCH, n_test);
  std::vector<uint8_t> img((size_t)n_train * IMG_BYTES);
  std::vector<int> lab(n_train);
  uint32_t h = 12345;
  for (auto& v : img) { h = h * 1664525u + 1013904223u; v = (uint8_t)(h >> 24); }
  for (int i = 0; i < n_train; ++i) lab[i] = i % NCLS;

  LeNetBuffers b;
  uint8_t* images = dalloc<uint8_t>(img.size());
  int* labels = dalloc<int>(n_train);
  check_hip(hipMemcpy(images, img.data(), img.size(), hipMemcpyHostToDevice), "copy images");
  check_hip(hipMemcpy(labels, lab.data(), lab.size() * sizeof(int), hipMemcpyHostToDevice), "copy labels");
  b.train_images = images;
  b.train_labels = labels;
  b.n_train = n_train;
  b.params = dalloc<float>(P_TOTAL);
  b.mom = dalloc<float>(P_TOTAL);
  b.pk = dalloc<bf16>(PK_TOTAL);
  b.act2 = dalloc<bf16>((size_t)rows * F0P);
  b.act2_rows = rows;
  b.act2T = dalloc<bf16>((size_t)F0P * MAX_TRAIN_BATCH);
  b.h1 = dalloc<bf16>((size_t)MAX_TRAIN_BATCH * 128);
  b.dact2 = dalloc<float>((size_t)MAX_TRAIN_BATCH * F0);
  b.dZ1T = dalloc<bf16>((size_t)DZ1_LD * MAX_TRAIN_BATCH);
  b.conv_slab = dalloc<float>((size_t)MAX_TRAIN_BATCH * CS);
  b.eval_part_floats = 2L * ((rows + FC_SPW - 1) / FC_SPW);
  b.eval_part = dalloc<float>((size_t)b.eval_part_floats);
  Stats* stats = dalloc<Stats>(2);
  b.train_stats = stats;
  b.eval_stats = stats + 1;
  b.round_ctr = dalloc<int>(4);

  // small random weights
  std::vector<float> p0(P_TOTAL);
  for (auto& v : p0) { h = h * 1664525u + 1013904223u; v = ((float)(h >> 8) / 16777216.f - 0.5f) * 0.1f; }
  check_hip(hipMemcpy(b.params, p0.data(), p0.size() * sizeof(float), hipMemcpyHostToDevice), "copy params");

  hipStream_t st;
  check_hip(hipStreamCreate(&st), "stream");
  {
    LeNetEngine eng(b, SgdConfig{}, 7u, true);
    eng.pack(st);
    // error paths
    try { eng.set_schedule({0, 128}, {128}); expect(false, "length mismatch accepted"); } catch (const std::invalid_argument&) {}
    try { eng.step(st, n_train - 10, 64, false); expect(false, "out-of-range batch accepted"); } catch (const std::invalid_argument&) {}
    eng.set_schedule({0, 128, 384, 896}, {128, 128, 33, 80});
    for (int rep = 0; rep < 2; ++rep) {       // eager and graph epochs, graph re-capture after a new schedule
      for (int use_graph = 0; use_graph < 2; ++use_graph)
        for (int ep = 0; ep < 2; ++ep) eng.run_epoch(st, use_graph != 0);
      eng.eval(st, images, labels, n_test);
      eng.set_schedule({0, 128, 384, 896}, {128, 128, 33, 80});
    }
    eng.set_schedule({}, {});
    eng.run_epoch(st, true);           // a rank that owns no batch this round
    check_hip(hipStreamSynchronize(st), "sync");
  }
  std::vector<float> p1(P_TOTAL);
  check_hip(hipMemcpy(p1.data(), b.params, p1.size() * sizeof(float), hipMemcpyDeviceToHost), "copy back");
  bool finite = true, moved = false;
  for (int i = 0; i < P_TOTAL; ++i) {
    finite &= std::isfinite(p1[i]);
    moved |= p1[i] != p0[i];
  }
  expect(finite, "non-finite parameters");
  expect(moved, "parameters did not move");
  Stats hs[2];
  check_hip(hipMemcpy(hs, stats, sizeof(hs), hipMemcpyDeviceToHost), "copy stats");
  expect(hs[1].count == n_test, "eval count");
  check_hip(hipStreamDestroy(st), "stream destroy");
  std::printf("lenet_engine_asan: %s (eval acc %.2f %%, %d failures)\n", failures ? "FAILED" : "ok",
              100.0 * hs[1].correct / std::max(1, hs[1].count), failures);
  return failures ? 1 : 0;
}
