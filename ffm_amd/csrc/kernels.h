// kernels.h -- host-side launch interface of the FFM HIP kernels (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace ffm {

// ceil(2^32 / d): n / d == mulhi(n, magic_div(d)) whenever n * d < 2^32 (core_common.h mdiv).
// Callers check it on the host (magic_div_ok): the engine's padded cell indices, and the
// learner's cell indices and coordinates, all stay below it for maps of <= 65,536 cells.
__host__ __device__ inline uint32_t magic_div(uint32_t d) { return (uint32_t)((0x100000000ull + d - 1) / d); }
// every n < n_end divides exactly by magic_div(d)
__host__ __device__ inline bool magic_div_ok(uint64_t n_end, uint32_t d) { return n_end * (uint64_t)d <= 0x100000000ull; }

struct CoreStepArgs {
    int H, W, HW;          // map shape
    uint32_t mW, mPW;      // magic_div(W), magic_div(W + 2): row of a cell index by one multiply-high
    int A;                 // agent slots per env (stride of pos)
    int K;                 // envs per workgroup
    long long E;           // envs on this device
    long long env_base;    // global id of env 0 (RNG key)
    uint16_t* pos;         // [E][A] cell indices
    int* cnt;              // [E]
    float* dff;            // [E][HW]
    int* episodes;         // [E] or nullptr
    unsigned long long* counters;  // [slots][4] agent_steps, exits, resets, steps (one slot per wave/block)
    const uint8_t* pmap;   // [(H+2)*(W+2)] padded map codes: 0 free, 2 blocked, 3 exit
    const void* psff;      // [(H+2)*(W+2)] padded SFF, f32 or f64
    float kS32, kD32;      // f32(-k_S), f32(k_D)
    double kS64;           // -k_S (float64 SFF path)
    float c0, c1;          // f32((1-decay)(1-diffuse)), f32(decay(1-diffuse)/|nb|)
    uint32_t key0, key1;   // Philox key (seed)
    uint32_t t;            // step index (Philox counter word 0)
    int auto_reset, N;     // re-place N agents when an env empties
    const uint16_t* free_list;  // [F] row-major free cells
    const uint16_t* free_padded;  // [F] the same cells as padded indices (x+1)*(W+2)+y+1
    int F;
    uint32_t* mt_np;       // [E][625] MT mode
    uint32_t* mt_py;       // [E][625]
    unsigned long long* dbg;  // diagnostic builds: [16] per-phase cycle sums (else unused)
    unsigned char* scratch;   // big maps: [blocks][scratch_stride] block state (else nullptr)
    size_t scratch_stride;
};

// Trajectory capture of the batched ffm_core step (ffm_engine_set_trajectory_capture):
// rows of {global env, episode, step in episode, count} + agent cells after every step.
struct CoreCapture {
    const int* envs;           // [n_sel] local env indices
    const int* phase;          // [n_sel] or nullptr
    int* state;                // [n_sel][3]: episode being logged, its steps so far, count after the last step
    int* meta;                 // [cap][4]
    uint16_t* cells;           // [cap][A]
    unsigned long long* n;     // rows appended (may pass cap: dropped)
    long long cap;
    int n_sel, period;
};

size_t core_wave_smem_bytes(int H, int W, int A, int F, bool mt, bool reset, int waves);
size_t core_block_smem_bytes(int H, int W, int A, int K, int F, bool f64, bool mt, bool reset);
hipError_t launch_core_wave(const CoreStepArgs& a, int nb, bool mt, int blocks, hipStream_t s);
int core_wave_blocks_per_cu(const CoreStepArgs& a, int nb, bool mt);
size_t core_lane_smem_bytes(int H, int W, int F, int waves);
hipError_t launch_core_lane(const CoreStepArgs& a, int nb, int blocks, hipStream_t s);
int core_lane_blocks_per_cu(const CoreStepArgs& a, int nb);
int core_lane_max_pairs_per_wave();
size_t core_group_smem_bytes(int H, int W, int F, int waves, int G = 4);
bool core_group_supported(int H, int W);
int core_group_max_iters();
int core_group_pick_envs(const CoreStepArgs& a, int nb, long long E, int cus);   // envs per group (2 or 4)
hipError_t launch_core_group(const CoreStepArgs& a, int nb, int blocks, hipStream_t s, int G);
int core_group_blocks_per_cu(const CoreStepArgs& a, int nb, int G);
size_t core_multi_smem_bytes(int H, int W, int F, int waves);
hipError_t launch_core_multi(const CoreStepArgs& a, int nb, int nsteps, int blocks, hipStream_t s);
int core_multi_blocks_per_cu(const CoreStepArgs& a, int nb);
hipError_t launch_core_block(const CoreStepArgs& a, int nb, bool f64, bool mt, int block, hipStream_t s);
hipError_t launch_core_reset(const CoreStepArgs& a, hipStream_t s, const uint8_t* mask = nullptr);
size_t core_big_scratch_bytes(int H, int W, int A, int F, bool mt);
hipError_t launch_core_block_reset(const CoreStepArgs& a, hipStream_t s, const uint8_t* mask = nullptr);
hipError_t launch_update_dff(const float* src, float* dst, long long E, int H, int W, int nb, float c0,
                             float c1, hipStream_t s);
hipError_t launch_core_capture_init(const CoreStepArgs& a, const CoreCapture& c, hipStream_t s);
hipError_t launch_core_capture(const CoreStepArgs& a, const CoreCapture& c, hipStream_t s);
hipError_t launch_np_expf(const float* x, float* y, long long n, hipStream_t s);

}  // namespace ffm
