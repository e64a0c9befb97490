// Mel features and Griffin-Lim on the GPU: the
// reference's src/utils/audio.py:45-151 (compute_mel_spectrogram,
// mel_to_audio), which call librosa 0.10 (STFT with a periodic Hann window,
// centre zero padding, Slaney mel filters, power_to_db, NNLS, Griffin-Lim).
//
// STFT / iSTFT frames are one workgroup each: the frame is gathered from the
// signal (coalesced, zero outside it), windowed, and transformed by a
// radix-2 Stockham FFT in LDS (ping-pong complex buffers, twiddles from a
// table computed in double precision on the host).  The STFT is HBM-light:
// a frame reads 4 KB of signal and writes 4 KB of spectrum, ~50 kFLOP, so
// the launch is latency-bound at the frame counts of an utterance; it is
// not reshaped into a DFT-GEMM.
//   mel features: frame -> FFT -> |X|^2 -> mel filters (per band a
//     contiguous bin range) -> [n_mels, frames]; then one workgroup per
//     utterance does power_to_db (ref = max, amin 1e-10, top_db 80) and the
//     [-1, 1] normalisation with LDS reductions.
//   Griffin-Lim: magnitudes from the mel by projected-gradient NNLS
//     (Nesterov-accelerated, X >= 0, from the clipped pseudo-inverse like
//     librosa.util.nnls's start), then n_iter x [iSTFT frames -> overlap-add
//     with the window-sum-square division -> STFT frames with the momentum
//     update of the phases]; the overlap-add is a gather (each sample sums
//     its <= n_fft / hop frames), so results are deterministic.
#include <cmath>
#include <cstring>
#include <vector>

#include "m2_common.h"

namespace m2 {
namespace dsp {

constexpr int NT = 256;  // threads per frame workgroup

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }

// In-LDS radix-2 Stockham FFT of N points (natural order in and out),
// a -> result in a or b (returned).  tw[k] = exp(-2 pi i k / N), k < N/2;
// INV: conjugated twiddles (unnormalised inverse).
template <int N, bool INV>
__device__ float2* fft_lds(float2* a, float2* b, const float2* __restrict__ tw) {
    float2* x = a;
    float2* y = b;
    for (int ns = 1; ns < N; ns <<= 1) {
        for (int j = threadIdx.x; j < N / 2; j += NT) {
            const int k = j & (ns - 1);
            float2 w = tw[k * (N / (2 * ns))];
            if (INV) w.y = -w.y;
            const float2 u = x[j], v = cmul(x[j + N / 2], w);
            const int o = ((j - k) << 1) + k;
            y[o] = make_float2(u.x + v.x, u.y + v.y);
            y[o + ns] = make_float2(u.x - v.x, u.y - v.y);
        }
        __syncthreads();
        float2* t = x;
        x = y;
        y = t;
    }
    return x;
}

// Frame t of utterance b: samples t*hop - N/2 + n (centre padding, zero
// outside [0, L)) times the window, into LDS as complex.
template <int N>
__device__ void load_frame(const float* __restrict__ y, int L, int hop, int t, const float* __restrict__ win, float2* a) {
    const int s0 = t * hop - N / 2;
    for (int n = threadIdx.x; n < N; n += NT) {
        const int i = s0 + n;
        a[n] = make_float2((i >= 0 && i < L) ? y[i] * win[n] : 0.f, 0.f);
    }
    __syncthreads();
}

// STFT to power, mel filters: mel[b, m, t] = sum_f W[m, f] |X_t[f]|^2
// (band m covers bins [lo[m], hi[m])).  Or the complex spectrum
// spec[b, t, f] (f <= N/2) when spec != null.
template <int N>
__global__ __launch_bounds__(NT) void stft_kernel(const float* __restrict__ y, int L, int hop, int frames,
                                                  const float* __restrict__ win, const float2* __restrict__ tw,
                                                  const float* __restrict__ W, const int* __restrict__ lo,
                                                  const int* __restrict__ hi, int n_mels, float* __restrict__ mel,
                                                  float2* __restrict__ spec) {
    __shared__ float2 a[N], b[N];
    __shared__ float P[N / 2 + 1];
    const int t = blockIdx.x, u = blockIdx.y;
    load_frame<N>(y + (size_t)u * L, L, hop, t, win, a);
    const float2* X = fft_lds<N, false>(a, b, tw);
    constexpr int F = N / 2 + 1;
    if (spec) {
        for (int f = threadIdx.x; f < F; f += NT) spec[((size_t)u * frames + t) * F + f] = X[f];
        return;
    }
    for (int f = threadIdx.x; f < F; f += NT) P[f] = X[f].x * X[f].x + X[f].y * X[f].y;
    __syncthreads();
    for (int m = threadIdx.x; m < n_mels; m += NT) {
        float s = 0.f;
        for (int f = lo[m]; f < hi[m]; ++f) s += W[(size_t)m * F + f] * P[f];
        mel[((size_t)u * n_mels + m) * frames + t] = s;
    }
}

__device__ float block_reduce(float v, bool is_max, float* red) {
    for (int o = 32; o > 0; o >>= 1) {
        const float w = __shfl_xor(v, o);
        v = is_max ? fmaxf(v, w) : fminf(v, w);
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[wv] = v;
    __syncthreads();
    v = red[0];
    for (int i = 1; i < nw; ++i) v = is_max ? fmaxf(v, red[i]) : fminf(v, red[i]);
    return v;
}

// power_to_db(ref=max, amin=1e-10, top_db=80) and 2 (x - min)/(max - min) - 1,
// in place over one utterance's [n_mels, frames] (one workgroup).
__global__ __launch_bounds__(1024) void db_norm_kernel(float* __restrict__ mel, int n) {
    __shared__ float red[16];
    float* x = mel + (size_t)blockIdx.x * n;
    float mx = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, x[i]);
    const float ref = block_reduce(mx, true, red);
    const float off = 10.f * log10f(fmaxf(1e-10f, ref));
    float lmax = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float v = 10.f * log10f(fmaxf(1e-10f, x[i])) - off;
        x[i] = v;
        lmax = fmaxf(lmax, v);
    }
    const float floor_db = block_reduce(lmax, true, red) - 80.f;
    float vmin = INFINITY, vmax2 = -INFINITY;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float v = fmaxf(x[i], floor_db);
        x[i] = v;
        vmin = fminf(vmin, v);
        vmax2 = fmaxf(vmax2, v);
    }
    const float lo = block_reduce(vmin, false, red), hi = block_reduce(vmax2, true, red);
    const float sc = 2.f / (hi - lo);
    for (int i = threadIdx.x; i < n; i += blockDim.x) x[i] = (x[i] - lo) * sc - 1.f;
}

// Griffin-Lim magnitudes (librosa.feature.inverse.mel_to_stft, power 2):
// X = librosa.util.nnls(W, M) for M = 10^(0.1 (x + 1) / 2), S = sqrt(X).
// librosa solves each block of kNnlsBlockBytes / (n_mels * 4) columns with
// scipy's L-BFGS-B (pgtol 1e-5) on (1 / block size) * 0.5 ||W X - M||^2 from
// X0 = max(0, pinv(W) M), and L-BFGS-B's first act is its convergence test
// at X0: the infinity norm of the projected gradient (g if g < 0, else
// min(x, g)).  For every mel in the reference's normalised range it passes
// (the scaled gradient at X0 is ~1e-7 or less), so librosa returns X0.  Two
// launches reproduce that exactly:
//   nnls_start_kernel  (one workgroup per frame): X0, the residual and the
//     scaled gradient in double, the frame's projected-gradient maximum;
//   nnls_finish_kernel (one per frame): the block's maximum; a converged
//     block stores sqrt(X0) - librosa's result - and a block L-BFGS-B would
//     iterate (mel far outside the normalised range) runs `iters` Nesterov
//     projected-gradient steps per frame from X0 instead, which reaches an
//     NNLS minimiser of the frame but not necessarily L-BFGS-B's (the
//     system is under-determined).
constexpr double kNnlsPgtol = 1e-5;            // scipy fmin_l_bfgs_b default
constexpr int kNnlsBlockBytes = 256 * 1024;    // librosa.util.utils.MAX_MEM_BLOCK
__host__ __device__ inline int nnls_block_cols(int n_mels) {
    const int c = kNnlsBlockBytes / (n_mels * 4);
    return c > 0 ? c : 1;
}

__global__ __launch_bounds__(NT) void nnls_start_kernel(const float* __restrict__ mel, int n_mels, int frames, int F,
                                                        const float* __restrict__ W, const float* __restrict__ Wp,
                                                        float* __restrict__ X0, float* __restrict__ pgmax) {
    extern __shared__ float sh[];
    float* M = sh;                                      // [n_mels]
    float* X = M + n_mels;                              // [F]
    // [n_mels] residual: at float offset n_mels + F rounded up to even (8-B aligned)
    double* r = reinterpret_cast<double*>(sh + ((n_mels + F + 1) & ~1));
    __shared__ double red[NT / 64];
    const int t = blockIdx.x, u = blockIdx.y;
    for (int m = threadIdx.x; m < n_mels; m += NT)
        M[m] = exp10f(0.1f * 0.5f * (mel[((size_t)u * n_mels + m) * frames + t] + 1.f));
    __syncthreads();
    for (int f = threadIdx.x; f < F; f += NT) {
        float s = 0.f;
        for (int m = 0; m < n_mels; ++m) s += Wp[(size_t)f * n_mels + m] * M[m];
        X[f] = fmaxf(s, 0.f);
        X0[((size_t)u * frames + t) * F + f] = X[f];
    }
    __syncthreads();
    for (int m = threadIdx.x; m < n_mels; m += NT) {
        double s = -(double)M[m];
        for (int f = 0; f < F; ++f) s += (double)W[(size_t)m * F + f] * (double)X[f];
        r[m] = s;
    }
    __syncthreads();
    const int bc = nnls_block_cols(n_mels), b0 = t / bc * bc;
    const double inv = 1.0 / ((double)n_mels * (double)min(bc, frames - b0));
    double mx = 0.0;
    for (int f = threadIdx.x; f < F; f += NT) {
        double g = 0.0;
        for (int m = 0; m < n_mels; ++m) g += (double)W[(size_t)m * F + f] * r[m];
        g *= inv;
        const double pg = g < 0.0 ? g : fmin((double)X[f], g);  // L-BFGS-B projgr, bound x >= 0
        mx = fmax(mx, fabs(pg));
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < NT / 64; ++w) mx = fmax(mx, red[w]);
        pgmax[(size_t)u * frames + t] = (float)mx;
    }
}

__global__ __launch_bounds__(NT) void nnls_finish_kernel(const float* __restrict__ mel, int n_mels, int frames, int F,
                                                         const float* __restrict__ W, float step, int iters,
                                                         const float* __restrict__ pgmax, float* __restrict__ S) {
    extern __shared__ float sh[];
    float* M = sh;              // [n_mels]
    float* r = M + n_mels;      // [n_mels] residual
    float* X = r + n_mels;      // [F]
    float* Yk = X + F;          // [F] extrapolated point
    __shared__ int conv;
    const int t = blockIdx.x, u = blockIdx.y;
    const int bc = nnls_block_cols(n_mels), b0 = t / bc * bc, b1 = min(frames, b0 + bc);
    float mx = 0.f;
    for (int k = b0 + threadIdx.x; k < b1; k += NT) mx = fmaxf(mx, pgmax[(size_t)u * frames + k]);
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
    if (threadIdx.x == 0) conv = 1;
    __syncthreads();
    if ((threadIdx.x & 63) == 0 && !((double)mx <= kNnlsPgtol)) conv = 0;
    __syncthreads();
    float* srow = S + ((size_t)u * frames + t) * F;  // holds X0 (nnls_start_kernel)
    if (conv || iters == 0) {  // librosa's result: X0
        for (int f = threadIdx.x; f < F; f += NT) srow[f] = sqrtf(srow[f]);
        return;
    }
    for (int m = threadIdx.x; m < n_mels; m += NT)
        M[m] = exp10f(0.1f * 0.5f * (mel[((size_t)u * n_mels + m) * frames + t] + 1.f));
    for (int f = threadIdx.x; f < F; f += NT) {
        X[f] = srow[f];
        Yk[f] = X[f];
    }
    __syncthreads();
    float tk = 1.f;
    for (int it = 0; it < iters; ++it) {
        for (int m = threadIdx.x; m < n_mels; m += NT) {
            float s = -M[m];
            for (int f = 0; f < F; ++f) s += W[(size_t)m * F + f] * Yk[f];
            r[m] = s;
        }
        __syncthreads();
        const float tn = 0.5f * (1.f + sqrtf(1.f + 4.f * tk * tk)), beta = (tk - 1.f) / tn;
        for (int f = threadIdx.x; f < F; f += NT) {
            float g = 0.f;
            for (int m = 0; m < n_mels; ++m) g += W[(size_t)m * F + f] * r[m];
            const float xn = fmaxf(Yk[f] - step * g, 0.f);
            Yk[f] = xn + beta * (xn - X[f]);
            X[f] = xn;
        }
        tk = tn;
        __syncthreads();
    }
    for (int f = threadIdx.x; f < F; f += NT) srow[f] = sqrtf(X[f]);
}

// iSTFT frame t: the spectrum S * angles (Hermitian-completed; the imaginary
// parts of DC and Nyquist dropped, as irfft does), inverse FFT / N, times
// the window -> fr[b, t, 0:N].
template <int N>
__global__ __launch_bounds__(NT) void istft_frame_kernel(const float* __restrict__ S, const float2* __restrict__ ang,
                                                         int frames, const float* __restrict__ win,
                                                         const float2* __restrict__ tw, float* __restrict__ fr) {
    __shared__ float2 a[N], b[N];
    constexpr int F = N / 2 + 1;
    const int t = blockIdx.x, u = blockIdx.y;
    const size_t row = ((size_t)u * frames + t) * F;
    for (int f = threadIdx.x; f < F; f += NT) {
        float2 c = ang[row + f];
        const float m = S[row + f];
        c = make_float2(c.x * m, c.y * m);
        if (f == 0 || f == N / 2) c.y = 0.f;
        a[f] = c;
        if (f > 0 && f < N / 2) a[N - f] = make_float2(c.x, -c.y);
    }
    __syncthreads();
    const float2* x = fft_lds<N, true>(a, b, tw);
    float* o = fr + ((size_t)u * frames + t) * N;
    for (int n = threadIdx.x; n < N; n += NT) o[n] = x[n].x * (1.f / N) * win[n];
}

// Overlap-add with the window-sum-square division (where it exceeds
// tiny(float32)), centre padding trimmed: y[b, i], i < hop (frames - 1).
template <int N>
__global__ __launch_bounds__(256) void ola_kernel(const float* __restrict__ fr, int frames, int hop,
                                                  const float* __restrict__ win, int Lout, float* __restrict__ y) {
    const int i = blockIdx.x * 256 + threadIdx.x, u = blockIdx.y;
    if (i >= Lout) return;
    const int p = i + N / 2;  // position in the untrimmed signal
    int t1 = p / hop;
    if (t1 > frames - 1) t1 = frames - 1;
    const int t0 = p >= N ? (p - N) / hop + 1 : 0;
    float s = 0.f, w2 = 0.f;
    for (int t = t0; t <= t1; ++t) {
        const int n = p - t * hop;
        s += fr[((size_t)u * frames + t) * N + n];
        w2 += win[n] * win[n];
    }
    y[(size_t)u * Lout + i] = w2 > 1.17549435e-38f ? s / w2 : s;
}

// STFT of the rebuilt signal and the Griffin-Lim phase update:
// angles = (X - m/(1+m) prev) / (|.| + tiny), prev = X.
template <int N>
__global__ __launch_bounds__(NT) void gl_update_kernel(const float* __restrict__ y, int L, int hop, int frames,
                                                       const float* __restrict__ win, const float2* __restrict__ tw,
                                                       float mom, float2* __restrict__ ang, float2* __restrict__ prev) {
    __shared__ float2 a[N], b[N];
    constexpr int F = N / 2 + 1;
    const int t = blockIdx.x, u = blockIdx.y;
    load_frame<N>(y + (size_t)u * L, L, hop, t, win, a);
    const float2* X = fft_lds<N, false>(a, b, tw);
    const size_t row = ((size_t)u * frames + t) * F;
    const float c = mom / (1.f + mom);
    for (int f = threadIdx.x; f < F; f += NT) {
        const float2 r = X[f], q = prev[row + f];
        float2 v = make_float2(r.x - c * q.x, r.y - c * q.y);
        const float inv = 1.f / (sqrtf(v.x * v.x + v.y * v.y) + 1.17549435e-38f);
        ang[row + f] = make_float2(v.x * inv, v.y * inv);
        prev[row + f] = r;
    }
}

// y /= max |y| per utterance (audio.py:146-147), one workgroup each.
__global__ __launch_bounds__(1024) void peak_norm_kernel(float* __restrict__ y, int L) {
    __shared__ float red[16];
    float* x = y + (size_t)blockIdx.x * L;
    float mx = 0.f;
    for (int i = threadIdx.x; i < L; i += blockDim.x) mx = fmaxf(mx, fabsf(x[i]));
    mx = block_reduce(mx, true, red);
    if (mx > 0.f)
        for (int i = threadIdx.x; i < L; i += blockDim.x) x[i] /= mx;
}

}  // namespace dsp
}  // namespace m2

// ---------------------------------------------------------------------------
// Host side: the per-configuration tables (window, twiddles, mel filters and
// their pseudo-inverse) live in one device allocation owned by m2_dsp.
struct m2_dsp {
    int sr, n_fft, hop, win_length, n_mels;
    float fmin, fmax;
    float* buf = nullptr;
    float *win, *W, *Wp;
    float2* tw;
    int *lo, *hi;
    float step;  // NNLS gradient step 1 / ||W||_2^2
};

namespace {
using namespace m2;

double hz_to_mel(double f) {  // librosa Slaney scale
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return f >= min_log_hz ? min_log_mel + std::log(f / min_log_hz) / logstep : f / f_sp;
}
double mel_to_hz(double m) {
    const double f_sp = 200.0 / 3, min_log_hz = 1000.0, min_log_mel = min_log_hz / f_sp, logstep = std::log(6.4) / 27.0;
    return m >= min_log_mel ? min_log_hz * std::exp(logstep * (m - min_log_mel)) : f_sp * m;
}

// Moore-Penrose pseudo-inverse of the [n_mels x F] filter matrix (full row
// rank): W^T (W W^T)^-1 by Gauss-Jordan on the small n_mels x n_mels Gram
// matrix, in double.
bool pinv_rows(const std::vector<double>& W, int R, int F, std::vector<double>* out) {
    std::vector<double> G((size_t)R * 2 * R, 0.0);
    for (int i = 0; i < R; ++i) {
        for (int j = 0; j < R; ++j) {
            double s = 0.0;
            for (int f = 0; f < F; ++f) s += W[(size_t)i * F + f] * W[(size_t)j * F + f];
            G[(size_t)i * 2 * R + j] = s;
        }
        G[(size_t)i * 2 * R + R + i] = 1.0;
    }
    for (int c = 0; c < R; ++c) {
        int p = c;
        for (int i = c + 1; i < R; ++i)
            if (std::fabs(G[(size_t)i * 2 * R + c]) > std::fabs(G[(size_t)p * 2 * R + c])) p = i;
        if (std::fabs(G[(size_t)p * 2 * R + c]) < 1e-300) return false;
        for (int k = 0; k < 2 * R; ++k) std::swap(G[(size_t)c * 2 * R + k], G[(size_t)p * 2 * R + k]);
        const double d = G[(size_t)c * 2 * R + c];
        for (int k = 0; k < 2 * R; ++k) G[(size_t)c * 2 * R + k] /= d;
        for (int i = 0; i < R; ++i)
            if (i != c) {
                const double e = G[(size_t)i * 2 * R + c];
                if (e != 0.0)
                    for (int k = 0; k < 2 * R; ++k) G[(size_t)i * 2 * R + k] -= e * G[(size_t)c * 2 * R + k];
            }
    }
    out->assign((size_t)F * R, 0.0);  // [F][R] = W^T Ginv
    for (int f = 0; f < F; ++f)
        for (int j = 0; j < R; ++j) {
            double s = 0.0;
            for (int i = 0; i < R; ++i) s += W[(size_t)i * F + f] * G[(size_t)i * 2 * R + R + j];
            (*out)[(size_t)f * R + j] = s;
        }
    return true;
}

int frames_of(const m2_dsp* d, int L) { return 1 + L / d->hop; }  // 1 + (L + 2 (n_fft/2) - n_fft) / hop

// X = librosa.util.nnls(W, M) -> S = sqrt(X) [B, T, F] (nnls_start_kernel /
// nnls_finish_kernel); pg: B * T floats of scratch.
int32_t nnls_magnitudes(const m2_dsp* d, const float* mel, int B, int T, int iters, float* S, float* pg,
                        hipStream_t st) {
    const int F = d->n_fft / 2 + 1;
    const dim3 grid(T, B);
    // M [n_mels] | X [F] floats, rounded up to an even count, then r [n_mels] doubles
    const size_t shs = (((size_t)d->n_mels + (size_t)F + 1) & ~(size_t)1) * sizeof(float) + (size_t)d->n_mels * sizeof(double);
    hipLaunchKernelGGL(dsp::nnls_start_kernel, grid, dim3(dsp::NT), shs, st, mel, d->n_mels, T, F, d->W, d->Wp, S, pg);
    M2_LAUNCHED("nnls_start_kernel");
    const size_t shf = (2 * (size_t)d->n_mels + 2 * (size_t)F) * sizeof(float);
    hipLaunchKernelGGL(dsp::nnls_finish_kernel, grid, dim3(dsp::NT), shf, st, mel, d->n_mels, T, F, d->W, d->step,
                       iters, pg, S);
    M2_LAUNCHED("nnls_finish_kernel");
    return M2_OK;
}
}  // namespace

extern "C" {

int32_t m2_dsp_create(int32_t sample_rate, int32_t n_fft, int32_t hop_length, int32_t win_length, int32_t n_mels,
                      float fmin, float fmax, void* stream, m2_dsp** out) {
    M2_CHECK_ARG(out && sample_rate > 0 && hop_length > 0 && n_mels > 0 && win_length > 0 && win_length <= n_fft &&
                     fmax > fmin && fmin >= 0,
                 "m2_dsp_create: bad argument");
    M2_CHECK_SHAPE(n_fft == 512 || n_fft == 1024 || n_fft == 2048, "m2_dsp_create: n_fft must be 512, 1024 or 2048");
    const int F = n_fft / 2 + 1;
    // periodic Hann of win_length, centred in n_fft (librosa pad_center)
    std::vector<float> win(n_fft, 0.f);
    const int lpad = (n_fft - win_length) / 2;
    for (int k = 0; k < win_length; ++k) win[lpad + k] = (float)(0.5 - 0.5 * std::cos(2.0 * M_PI * k / win_length));
    std::vector<float> tw(n_fft);  // n_fft/2 complex
    for (int k = 0; k < n_fft / 2; ++k) {
        tw[2 * k] = (float)std::cos(-2.0 * M_PI * k / n_fft);
        tw[2 * k + 1] = (float)std::sin(-2.0 * M_PI * k / n_fft);
    }
    // Slaney mel filters with area normalisation (librosa.filters.mel, htk=False, norm='slaney')
    std::vector<double> mel_f(n_mels + 2);
    const double m0 = hz_to_mel(fmin), m1 = hz_to_mel(fmax);
    for (int i = 0; i < n_mels + 2; ++i) mel_f[i] = mel_to_hz(m0 + (m1 - m0) * i / (n_mels + 1));
    std::vector<double> Wd((size_t)n_mels * F, 0.0);
    std::vector<int> lo(n_mels, F), hi(n_mels, 0);
    for (int i = 0; i < n_mels; ++i) {
        const double enorm = 2.0 / (mel_f[i + 2] - mel_f[i]);
        for (int f = 0; f < F; ++f) {
            const double hz = (double)f * sample_rate / n_fft;
            const double lower = (hz - mel_f[i]) / (mel_f[i + 1] - mel_f[i]);
            const double upper = (mel_f[i + 2] - hz) / (mel_f[i + 2] - mel_f[i + 1]);
            const double w = std::max(0.0, std::min(lower, upper)) * enorm;
            Wd[(size_t)i * F + f] = (double)(float)w;
            if (w > 0) {
                lo[i] = std::min(lo[i], f);
                hi[i] = std::max(hi[i], f + 1);
            }
        }
        if (hi[i] < lo[i]) lo[i] = hi[i] = 0;
    }
    std::vector<double> Pd;
    M2_CHECK_SHAPE(pinv_rows(Wd, n_mels, F, &Pd), "m2_dsp_create: mel filter matrix is rank deficient");
    // ||W||_2^2 = largest eigenvalue of W W^T (power iteration)
    std::vector<double> v(n_mels, 1.0), wv(F), nv(n_mels);
    double lam = 0.0;
    for (int it = 0; it < 200; ++it) {
        for (int f = 0; f < F; ++f) {
            double s = 0.0;
            for (int i = 0; i < n_mels; ++i) s += Wd[(size_t)i * F + f] * v[i];
            wv[f] = s;
        }
        double nrm = 0.0;
        for (int i = 0; i < n_mels; ++i) {
            double s = 0.0;
            for (int f = 0; f < F; ++f) s += Wd[(size_t)i * F + f] * wv[f];
            nv[i] = s;
            nrm += s * s;
        }
        nrm = std::sqrt(nrm);
        lam = nrm;
        for (int i = 0; i < n_mels; ++i) v[i] = nv[i] / nrm;
    }
    auto* d = new m2_dsp();
    d->sr = sample_rate;
    d->n_fft = n_fft;
    d->hop = hop_length;
    d->win_length = win_length;
    d->n_mels = n_mels;
    d->fmin = fmin;
    d->fmax = fmax;
    d->step = (float)(1.0 / lam);
    const size_t nw = n_fft, ntw = n_fft, nW = (size_t)n_mels * F, nP = (size_t)F * n_mels, nl = 2 * (size_t)n_mels;
    std::vector<float> host(nw + ntw + nW + nP + nl, 0.f);
    std::copy(win.begin(), win.end(), host.begin());
    std::copy(tw.begin(), tw.end(), host.begin() + nw);
    for (size_t i = 0; i < nW; ++i) host[nw + ntw + i] = (float)Wd[i];
    for (size_t i = 0; i < nP; ++i) host[nw + ntw + nW + i] = (float)Pd[i];
    std::memcpy(&host[nw + ntw + nW + nP], lo.data(), n_mels * sizeof(int));
    std::memcpy(&host[nw + ntw + nW + nP + n_mels], hi.data(), n_mels * sizeof(int));
    hipError_t e = hipMalloc(&d->buf, host.size() * sizeof(float));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d->buf, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        if (d->buf) (void)hipFree(d->buf);
        delete d;
        return hip_status(e, "m2_dsp_create: upload");
    }
    d->win = d->buf;
    d->tw = reinterpret_cast<float2*>(d->buf + nw);
    d->W = d->buf + nw + ntw;
    d->Wp = d->W + nW;
    d->lo = reinterpret_cast<int*>(d->Wp + nP);
    d->hi = d->lo + n_mels;
    *out = d;
    return M2_OK;
}

int32_t m2_dsp_destroy(m2_dsp* d) {
    if (!d) return M2_OK;
    const hipError_t e = hipFree(d->buf);
    delete d;
    return e == hipSuccess ? M2_OK : hip_status(e, "m2_dsp_destroy");
}

int32_t m2_dsp_frames(const m2_dsp* d, int32_t L) { return d && L >= 0 ? frames_of(d, L) : -1; }

int32_t m2_stft(const m2_dsp* d, const float* audio, int32_t B, int32_t L, void* out_spec, void* stream) {
    M2_CHECK_ARG(d && audio && out_spec && B >= 0 && L > 0, "m2_stft: bad argument");
    if (B == 0) return M2_OK;
    const int T = frames_of(d, L);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid(T, B);
#define M2_STFT(NN)                                                                                                     \
    hipLaunchKernelGGL((dsp::stft_kernel<NN>), grid, dim3(dsp::NT), 0, st, audio, L, d->hop, T, d->win, d->tw, d->W, \
                       d->lo, d->hi, d->n_mels, nullptr, static_cast<float2*>(out_spec))
    if (d->n_fft == 512) M2_STFT(512);
    else if (d->n_fft == 1024) M2_STFT(1024);
    else M2_STFT(2048);
#undef M2_STFT
    M2_LAUNCHED("stft_kernel");
    return M2_OK;
}

int32_t m2_mel_spectrogram(const m2_dsp* d, const float* audio, int32_t B, int32_t L, float* out_mel, void* stream) {
    M2_CHECK_ARG(d && audio && out_mel && B >= 0 && L > 0, "m2_mel_spectrogram: bad argument");
    if (B == 0) return M2_OK;
    const int T = frames_of(d, L);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid(T, B);
#define M2_MEL(NN)                                                                                                      \
    hipLaunchKernelGGL((dsp::stft_kernel<NN>), grid, dim3(dsp::NT), 0, st, audio, L, d->hop, T, d->win, d->tw, d->W, \
                       d->lo, d->hi, d->n_mels, out_mel, nullptr)
    if (d->n_fft == 512) M2_MEL(512);
    else if (d->n_fft == 1024) M2_MEL(1024);
    else M2_MEL(2048);
#undef M2_MEL
    M2_LAUNCHED("stft_kernel(mel)");
    hipLaunchKernelGGL(dsp::db_norm_kernel, dim3(B), dim3(1024), 0, st, out_mel, d->n_mels * T);
    M2_LAUNCHED("db_norm_kernel");
    return M2_OK;
}

size_t m2_mel_to_magnitude_workspace_bytes(const m2_dsp* d, int32_t B, int32_t T) {
    if (!d || B < 0 || T < 0) return 0;
    return ((size_t)B * T * sizeof(float) + 255) / 256 * 256 + 256;
}

int32_t m2_mel_to_magnitude(const m2_dsp* d, const float* mel, int32_t B, int32_t T, int32_t nnls_iters,
                            float* out_mag, void* workspace, size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(d && mel && out_mag && B >= 0 && T >= 0 && nnls_iters >= 0, "m2_mel_to_magnitude: bad argument");
    if (B == 0 || T == 0) return M2_OK;
    Carve c(workspace, workspace_bytes);
    float* pg = c.take<float>((size_t)B * T);
    if (!c.ok) return fail(M2_E_WORKSPACE, "m2_mel_to_magnitude: workspace too small");
    return nnls_magnitudes(d, mel, B, T, nnls_iters, out_mag, pg, static_cast<hipStream_t>(stream));
}

size_t m2_griffin_lim_workspace_bytes(const m2_dsp* d, int32_t B, int32_t T) {
    if (!d || B < 0 || T < 0) return 0;
    const int F = d->n_fft / 2 + 1, Lout = d->hop * (T > 0 ? T - 1 : 0);
    Sizer s;
    s.take<float>((size_t)B * T * F);           // magnitudes
    s.take<float2>((size_t)B * T * F);          // angles
    s.take<float2>((size_t)B * T * F);          // previous rebuilt spectrum
    s.take<float>((size_t)B * T * d->n_fft);    // windowed inverse frames
    s.take<float>((size_t)B * (Lout > 0 ? Lout : 1));  // the signal of each iteration
    s.take<float>((size_t)B * T);               // NNLS: per-frame projected-gradient maxima
    return s.off + 256;
}

// mag: if non-null the magnitudes [B, T, F] are taken from it (no mel / NNLS);
// else they come from mel [B, n_mels, T] (normalised dB, audio.py:128-132).
int32_t m2_griffin_lim(const m2_dsp* d, const float* mel, const float* mag, const void* init_angles, int32_t B,
                       int32_t T, int32_t n_iter, float momentum, int32_t nnls_iters, float* out_audio,
                       void* workspace, size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(d && (mel || mag) && init_angles && out_audio && B >= 0 && T >= 1 && n_iter >= 0 && nnls_iters >= 0,
                 "m2_griffin_lim: bad argument");
    M2_CHECK_SHAPE(T >= 2, "m2_griffin_lim: need at least 2 frames");
    if (B == 0) return M2_OK;
    const int N = d->n_fft, F = N / 2 + 1, Lout = d->hop * (T - 1);
    Carve c(workspace, workspace_bytes);
    float* S = c.take<float>((size_t)B * T * F);
    float2* ang = c.take<float2>((size_t)B * T * F);
    float2* prev = c.take<float2>((size_t)B * T * F);
    float* fr = c.take<float>((size_t)B * T * N);
    float* y = c.take<float>((size_t)B * Lout);
    float* pgw = mag ? nullptr : c.take<float>((size_t)B * T);
    if (!c.ok) return fail(M2_E_WORKSPACE, "m2_griffin_lim: workspace too small");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 fgrid(T, B);
    if (mag) {
        M2_HIP(hipMemcpyAsync(S, mag, (size_t)B * T * F * sizeof(float), hipMemcpyDeviceToDevice, st));
    } else {
        int32_t rc;
        if ((rc = nnls_magnitudes(d, mel, B, T, nnls_iters, S, pgw, st))) return rc;
    }
    M2_HIP(hipMemcpyAsync(ang, init_angles, (size_t)B * T * F * sizeof(float2), hipMemcpyDeviceToDevice, st));
    M2_HIP(hipMemsetAsync(prev, 0, (size_t)B * T * F * sizeof(float2), st));
    const dim3 ogrid(cdiv(Lout, 256), B);
    auto istft = [&](float* dst) -> int32_t {
#define M2_ISTFT(NN)                                                                                              \
    do {                                                                                                          \
        hipLaunchKernelGGL((dsp::istft_frame_kernel<NN>), fgrid, dim3(dsp::NT), 0, st, S, ang, T, d->win, d->tw, fr); \
        hipLaunchKernelGGL((dsp::ola_kernel<NN>), ogrid, dim3(256), 0, st, fr, T, d->hop, d->win, Lout, dst);       \
    } while (0)
        if (N == 512) M2_ISTFT(512);
        else if (N == 1024) M2_ISTFT(1024);
        else M2_ISTFT(2048);
#undef M2_ISTFT
        M2_LAUNCHED("istft");
        return M2_OK;
    };
    for (int it = 0; it < n_iter; ++it) {
        int32_t rc = istft(y);
        if (rc) return rc;
#define M2_GLU(NN)                                                                                                   \
    hipLaunchKernelGGL((dsp::gl_update_kernel<NN>), fgrid, dim3(dsp::NT), 0, st, y, Lout, d->hop, T, d->win, d->tw, \
                       momentum, ang, prev)
        if (N == 512) M2_GLU(512);
        else if (N == 1024) M2_GLU(1024);
        else M2_GLU(2048);
#undef M2_GLU
        M2_LAUNCHED("gl_update_kernel");
    }
    int32_t rc = istft(out_audio);
    if (rc) return rc;
    if (mel) {  // mel_to_audio's peak normalisation (audio.py:146-147); not for the bare Griffin-Lim
        hipLaunchKernelGGL(dsp::peak_norm_kernel, dim3(B), dim3(1024), 0, st, out_audio, Lout);
        M2_LAUNCHED("peak_norm_kernel");
    }
    return M2_OK;
}

}  // extern "C"
