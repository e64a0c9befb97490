// Shared helpers for the m2-tts gfx950 kernels and the C-ABI layer.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/m2tts_hip.h"

namespace m2 {

constexpr int kWave = 64;            // CDNA wavefront
constexpr float kLnEps = 1e-5f;      // nn.LayerNorm / BatchNorm1d default eps
constexpr float kLeaky = 0.1f;       // F.leaky_relu slope used by the vocoder
constexpr float kMaskFill = -1e9f;   // components.py:81 (masked_fill_ value)

enum Act : int { ACT_NONE = 0, ACT_LEAKY = 1, ACT_TANH = 2, ACT_RELU = 3, ACT_SOFTPLUS = 4 };

void set_error(const std::string& msg);

// Developer switches (M2_* environment variables: A/B comparisons and tests
// force one code path).  Read into this table when the library loads, again
// at every m2_model_create and by m2_reload_switches() - never per call.
// 0 (or -1 where 0 is a valid choice) = the default rule.
struct Switches {
    int dur_rb = 0;           // M2_DUR_RB=1|2: duration tiles of one / two row blocks
    int dur_count = -1;       // M2_DUR_COUNT=0|1: frame count fused into the duration kernel
    int speculative = 1;      // M2_SPECULATIVE=0: host-side T only
    bool tf_chain = true;     // M2_TF_CHAIN=0: separate ln_gemm launches
    bool tf_layer = true;     // M2_TF_LAYER=0: three-launch transformer layers
    bool tf_unfused = false;  // M2_TF_UNFUSED: five-linear layers (handle creation)
    int tf_waves = 0;         // M2_TF_WAVES=4|8
    int tfl_rb = 0;           // M2_TFL_RB=1|2|4
    int tfl_first_rb = 0;     // M2_TFL_FIRST_RB=1|2|4
    int tfl_rb_masked = 0;    // M2_TFL_RB_MASKED=1|2|4: rows per tile of the masked (encoder) launches
    int tfl_rb_unmasked = 0;  // M2_TFL_RB_UNMASKED=1|2|4: rows per tile of the unmasked (decoder) launches
    int tfl_qs2 = -1;         // M2_TFL_QS2=0|2|3|4|12
    int att_qt = 0;           // M2_ATT_QT
    bool att_f32 = false;     // M2_ATT_F32
    bool voc_perlayer = false;  // M2_VOCODER_PERLAYER (handle creation)
    bool voc_f32 = false;       // M2_VOC_F32 (handle creation)
    bool voc_tail_x3 = false;   // M2_VOC_TAIL_X3 (handle creation)
    bool voc_mid_x3 = false;    // M2_VOC_MID_X3 (handle creation)
    int voc_plan = -1;          // M2_VOC_PLAN
    int f32_mt = 2;             // M2_F32_MT=0|1|2|3: the stage1 exact-f32 16-wave tiling's mid / tail / both as 8-wave
                                // half windows (default 2: the tail, r06z3_mt.txt); 4: 2 + the mid's items halved
    bool f32_pair = true;       // M2_F32_PAIR=0: the stage1 exact-f32 tail's 8-channel layers phase by phase
    int x3_head_prio = 0;       // M2_X3_HEAD_PRIO=1: the split head's younger waves at higher issue priority
    bool f32_comp = true;       // M2_F32_COMP=0: the stage1 exact-f32 head's input conv as its own layer
    int midp_nch = 0;           // M2_MIDP_NCH: the stage1 mid's strip length in 16-column chunks (0: by grid)
    int tailp_nch = 0;          // M2_TAILP_NCH: strip length in 16-column chunks (0: by grid)
    bool tailp_seven = false;   // M2_TAILP_SEVEN
    int tailp2_nch = 0;         // M2_TAILP2_NCH: the same for the stage2 tail
    bool tailp2_seven = false;  // M2_TAILP2_SEVEN
    bool head_inconv = false;   // M2_HEAD_INCONV
    int s2_mid_alt = -1;        // M2_S2_MID_ALT=0|1: the 30- / 33-position stage2 mid (-1: by grid)
    int s2_head_tf = 0;         // M2_S2_HEAD_TF=16|19|24|27 (M2_S2_HEAD_TF16: 16)
    int redo_grid = -1;         // M2_REDO_GRID: workgroups of the guarded redo launch (-1: one per CU)
    bool redo_launch = false;   // M2_REDO_LAUNCH: the guarded exact-f32 launch also where the tail redoes locally
    bool dur_split = true;      // M2_DUR_SPLIT=0: the duration convs on the exact-f32 MFMA always
    bool dur_pers = true;       // M2_DUR_PERS=0: one duration tile per workgroup at every grid size
};
const Switches& sw();
void reload_switches();

// Status helpers: every C entry point returns through these.
int32_t fail(int32_t code, const char* what);
int32_t hip_status(hipError_t e, const char* where);

#define M2_CHECK_ARG(cond, msg)                      \
    do {                                             \
        if (!(cond)) return ::m2::fail(M2_E_ARG, msg); \
    } while (0)
#define M2_CHECK_SHAPE(cond, msg)                      \
    do {                                               \
        if (!(cond)) return ::m2::fail(M2_E_SHAPE, msg); \
    } while (0)
#define M2_HIP(expr)                                                   \
    do {                                                               \
        hipError_t _e = (expr);                                        \
        if (_e != hipSuccess) return ::m2::hip_status(_e, #expr);      \
    } while (0)
// After a kernel launch: surface launch-configuration errors immediately.
#define M2_LAUNCHED(name)                                              \
    do {                                                               \
        hipError_t _e = hipGetLastError();                             \
        if (_e != hipSuccess) return ::m2::hip_status(_e, name);       \
    } while (0)

__device__ __forceinline__ float apply_act(float v, int act) {
    if (act == ACT_LEAKY) return v > 0.f ? v : v * kLeaky;
    if (act == ACT_TANH) return tanhf(v);
    if (act == ACT_RELU) return v > 0.f ? v : 0.f;
    if (act == ACT_SOFTPLUS) return v > 20.f ? v : log1pf(expf(v));  // F.softplus(beta=1, threshold=20)
    return v;
}

template <int ACT>
__device__ __forceinline__ float act_t(float v) {
    if constexpr (ACT == ACT_LEAKY) return fmaxf(v, v * kLeaky);  // == (v > 0 ? v : 0.1v) for 0 < slope < 1
    else if constexpr (ACT == ACT_TANH) return tanhf(v);
    else if constexpr (ACT == ACT_RELU) return v > 0.f ? v : 0.f;
    else return v;
}

// Device-resident frame count of a speculatively launched back half
// (m2_inference with a known capacity, m2_inference_back_dev): the launch's
// grid covers `cap` frames; the kernels read T_max from the device word the
// length regulator (or the ranks' all-reduce) wrote and use T = max(1, T_max)
// (tts_model.py:158-160), or 0 - nothing to do - when T exceeds the capacity
// (the host then re-runs the back half for the real T).
__device__ __forceinline__ int dev_frames(const int32_t* p, int cap) {
    const int t = max(1, *p);
    return t <= cap ? t : 0;
}

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace (256-B aligned carves).
struct Carve {
    char* base;
    size_t cap;
    size_t off = 0;
    bool ok = true;
    Carve(void* p, size_t n) : base(static_cast<char*>(p)), cap(n) {}
    template <typename T>
    T* take(size_t count) {
        size_t o = align_up(off, 256);
        size_t n = count * sizeof(T);
        if (o + n > cap || base == nullptr) { ok = false; off = o + n; return nullptr; }
        off = o + n;
        return reinterpret_cast<T*>(base + o);
    }
};

// Byte counter with the same carve rule (for m2_workspace_bytes).
struct Sizer {
    size_t off = 0;
    template <typename T>
    T* take(size_t count) { off = align_up(off, 256) + count * sizeof(T); return nullptr; }
};

// nn.LayerNorm statistics of one row, one wave per row: two-pass mean and
// biased variance, lane-strided sums, xor-shuffle reductions.  Shared by
// layer_norm_kernel and the duration kernel's fused encoder LayerNorm so the
// two give identical bits.
__device__ __forceinline__ void ln_row_stats(const float* xr, int K, int lane, float& mean, float& rstd) {
    // explicit roundings: no context-dependent fma contraction between the
    // two kernels that use this
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s = __fadd_rn(s, xr[k]);
    for (int o = 32; o > 0; o >>= 1) s = __fadd_rn(s, __shfl_xor(s, o));
    mean = __fdiv_rn(s, (float)K);
    float v = 0.f;
    for (int k = lane; k < K; k += 64) {
        const float d = __fsub_rn(xr[k], mean);
        v = __fmaf_rn(d, d, v);
    }
    for (int o = 32; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o));
    rstd = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(__fdiv_rn(v, (float)K), kLnEps)));
}

// ln_row_stats on a row already in registers: x[q] = row[lane + 64 q] for
// lane + 64 q < K (the same additions in the same order).
template <int KP>
__device__ __forceinline__ void ln_row_stats_regs(const float (&x)[KP], int K, int lane, float& mean, float& rstd) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < KP; ++q)
        if (lane + 64 * q < K) s = __fadd_rn(s, x[q]);
    for (int o = 32; o > 0; o >>= 1) s = __fadd_rn(s, __shfl_xor(s, o));
    mean = __fdiv_rn(s, (float)K);
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < KP; ++q)
        if (lane + 64 * q < K) {
            const float d = __fsub_rn(x[q], mean);
            v = __fmaf_rn(d, d, v);
        }
    for (int o = 32; o > 0; o >>= 1) v = __fadd_rn(v, __shfl_xor(v, o));
    rstd = __fdiv_rn(1.0f, __fsqrt_rn(__fadd_rn(__fdiv_rn(v, (float)K), kLnEps)));
}

__device__ __forceinline__ float ln_apply(float x, float mean, float rstd, float g, float b) {
    return __fmaf_rn(__fmul_rn(__fsub_rn(x, mean), rstd), g, b);
}

}  // namespace m2
