// Probe: cost of handing a small payload from one workgroup to another inside one launch (VERDICT r4 item 5:
// "measure the hand-off cost before discarding the split-sample LeNet design").
//
// Two single-wave workgroups ping-pong R times: the producer stores a payload (PAY floats, the LeNet fc1
// activation / gradient size is 120-400) with plain vector stores, publishes a round counter with an
// agent-scope release store; the consumer polls it with agent-scope acquire loads, reads the payload, and
// answers on a second counter the same way.  One round = two hand-offs.  Placements: the pair on the same XCD
// (blocks 0 and 8: workgroups are dealt to the 8 XCDs round-robin) or on different XCDs (blocks 0 and 1).
// Every poll loop is bounded (no hang if a partner is never scheduled); all stores are vector stores.
//
//   hipcc -O3 --offload-arch=gfx950 tools/probes/l2_handoff.hip -o /tmp/l2_handoff && /tmp/l2_handoff
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int MAXPOLL = 1 << 22;

__global__ __launch_bounds__(64) void pingpong(float* payload, int* ping, int* pong, int rounds, int pay, int prod,
                                               int cons, long long* out, int* err) {
  const int b = blockIdx.x, lane = threadIdx.x;
  if (b != prod && b != cons) return;
  if (b == prod) {
    const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 1; i <= rounds; ++i) {
      for (int k = lane; k < pay; k += 64) payload[k] = (float)(i * 1000 + k);
      __syncthreads();
      if (lane == 0) __hip_atomic_store(ping, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      int n = 0;
      if (lane == 0)
        while (__hip_atomic_load(pong, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != i && ++n < MAXPOLL) {}
      n = __shfl(n, 0);
      if (n >= MAXPOLL) { if (lane == 0) atomicAdd(err, 1); return; }
    }
    const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
  } else {
    float acc = 0.f;
    for (int i = 1; i <= rounds; ++i) {
      int n = 0;
      if (lane == 0)
        while (__hip_atomic_load(ping, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != i && ++n < MAXPOLL) {}
      n = __shfl(n, 0);
      if (n >= MAXPOLL) { if (lane == 0) atomicAdd(err, 1); return; }
      __syncthreads();
      for (int k = lane; k < pay; k += 64) acc += __hip_atomic_load(payload + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane == 0) __hip_atomic_store(pong, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) out[2] = (long long)acc;   // keeps the payload reads
  }
}

int main() {
  float* payload;
  int *ping, *pong, *err;
  long long* out;
  hipMalloc(&payload, 4096 * sizeof(float));
  hipMalloc(&ping, 256);
  hipMalloc(&pong, 256);
  hipMalloc(&err, sizeof(int));
  hipMalloc(&out, 4 * sizeof(long long));
  const int rounds = 2000;
  struct Cfg { const char* name; int prod, cons, grid; };
  const Cfg cfgs[] = {{"same XCD (blocks 0, 8)", 0, 8, 9}, {"other XCD (blocks 0, 1)", 0, 1, 2}};
  const int pays[] = {0, 120, 400, 1600};
  for (const Cfg& c : cfgs) {
    for (int pay : pays) {
      for (int rep = 0; rep < 2; ++rep) {   // first run warms the caches / clocks
        hipMemset(ping, 0, 256);
        hipMemset(pong, 0, 256);
        hipMemset(err, 0, sizeof(int));
        hipMemset(out, 0, 4 * sizeof(long long));
        hipLaunchKernelGGL(pingpong, dim3(c.grid), dim3(64), 0, 0, payload, ping, pong, rounds, pay, c.prod, c.cons,
                           out, err);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
      }
      long long h[4];
      int e;
      hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
      hipMemcpy(&e, err, sizeof(int), hipMemcpyDeviceToHost);
      // one round = two hand-offs; s_memrealtime ticks at 100 MHz
      printf("{\"placement\": \"%s\", \"payload_floats\": %d, \"rounds\": %d, \"cycles_per_handoff\": %.0f, "
             "\"ns_per_handoff\": %.0f, \"timeouts\": %d}\n",
             c.name, pay, rounds, (double)h[0] / (2.0 * rounds), (double)h[1] * 10.0 / (2.0 * rounds), e);
    }
  }
  return 0;
}
