// C-ABI runtime: weight table, model handle, stage orchestration.
// See include/m2tts_hip.h for the contract of every entry point.
#include <immintrin.h>

#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "m2_common.h"
#include "transformer_fused.h"
#include "transformer_layer.h"
#include "vocoder_fused.h"

namespace m2 {

namespace {
// The published switch table: an immutable snapshot behind an atomic
// pointer.  reload_switches() (library load, every m2_model_create,
// m2_reload_switches) builds a new one and publishes it only when the
// environment changed; a reader sees one whole snapshot, never a table half
// rewritten by a concurrent creation.  Superseded snapshots are kept (a few
// hundred bytes per environment change), so a reference taken by sw() stays
// valid.  The table is process-wide: creating a handle under a changed
// environment changes the switches of every handle from its next call on.
std::atomic<const Switches*> g_swp{nullptr};
std::mutex g_sw_mu;
int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoi(e) : dflt;
}
bool env_set(const char* name) { return std::getenv(name) != nullptr; }
bool env_on(const char* name, bool dflt) {  // unset / empty -> dflt, else != "0"
    const char* e = std::getenv(name);
    return (e && *e) ? std::atoi(e) != 0 : dflt;
}
// reloaded when the library loads
const bool g_sw_loaded = (reload_switches(), true);
}  // namespace

const Switches& sw() { return *g_swp.load(std::memory_order_acquire); }

void reload_switches() {
    // zeroed storage, so the padding compares equal between snapshots
    void* raw = std::calloc(1, sizeof(Switches));
    if (!raw) return;  // keep the current table
    Switches& s = *new (raw) Switches();
    const int rb = env_int("M2_DUR_RB", 0);
    s.dur_rb = (rb == 1 || rb == 2) ? rb : 0;
    s.dur_count = std::getenv("M2_DUR_COUNT") && *std::getenv("M2_DUR_COUNT") ? (env_int("M2_DUR_COUNT", 0) != 0) : -1;
    s.speculative = env_on("M2_SPECULATIVE", true) ? 1 : 0;
    s.tf_chain = env_on("M2_TF_CHAIN", true);
    s.tf_layer = env_on("M2_TF_LAYER", true);
    s.tf_unfused = env_set("M2_TF_UNFUSED");
    const int tw = env_int("M2_TF_WAVES", 0);
    s.tf_waves = (tw == 4 || tw == 8) ? tw : 0;
    auto rb124 = [](int v) { return (v == 1 || v == 2 || v == 4) ? v : 0; };
    const int trb = env_int("M2_TFL_RB", 0);
    s.tfl_rb = rb124(trb);
    s.tfl_first_rb = rb124(env_int("M2_TFL_FIRST_RB", 0));
    s.tfl_rb_masked = rb124(env_int("M2_TFL_RB_MASKED", 0));
    s.tfl_rb_unmasked = rb124(env_int("M2_TFL_RB_UNMASKED", 0));
    if (const char* e = std::getenv("M2_TFL_QS2"); e && *e) {
        const int v = std::atoi(e);
        s.tfl_qs2 = (v == 2 || v == 3 || v == 4 || v == 12) ? v : 0;
    }
    s.att_qt = env_int("M2_ATT_QT", 0);
    if (const char* e = std::getenv("M2_ATT_F32")) s.att_f32 = *e && *e != '0';
    s.voc_perlayer = env_set("M2_VOCODER_PERLAYER");
    s.voc_f32 = env_set("M2_VOC_F32");
    s.voc_tail_x3 = env_set("M2_VOC_TAIL_X3");
    s.voc_mid_x3 = env_set("M2_VOC_MID_X3");
    s.voc_plan = env_int("M2_VOC_PLAN", -1);
    s.f32_mt = env_int("M2_F32_MT", 2);
    s.f32_pair = env_int("M2_F32_PAIR", 1) != 0;
    s.f32_comp = env_int("M2_F32_COMP", 1) != 0;
    s.x3_head_prio = env_int("M2_X3_HEAD_PRIO", 0);
    const int mn = env_int("M2_MIDP_NCH", 0);
    s.midp_nch = mn > 0 ? mn : 0;
    const int tn = env_int("M2_TAILP_NCH", 0);
    s.tailp_nch = tn > 0 ? tn : 0;
    s.tailp_seven = env_set("M2_TAILP_SEVEN");
    s.tailp2_nch = env_int("M2_TAILP2_NCH", 0);
    s.tailp2_seven = env_set("M2_TAILP2_SEVEN");
    s.head_inconv = env_set("M2_HEAD_INCONV");
    const int malt = env_int("M2_S2_MID_ALT", -1);
    s.s2_mid_alt = (malt == 0 || malt == 1) ? malt : -1;
    const int htf = env_int("M2_S2_HEAD_TF", env_set("M2_S2_HEAD_TF16") ? 16 : 0);
    s.s2_head_tf = (htf == 16 || htf == 19 || htf == 24 || htf == 27) ? htf : 0;
    s.redo_grid = env_int("M2_REDO_GRID", -1);
    s.redo_launch = env_set("M2_REDO_LAUNCH");
    s.dur_split = env_on("M2_DUR_SPLIT", true);
    s.dur_pers = env_on("M2_DUR_PERS", true);
    std::lock_guard<std::mutex> lk(g_sw_mu);
    const Switches* cur = g_swp.load(std::memory_order_relaxed);
    if (cur && std::memcmp(cur, &s, sizeof(Switches)) == 0) {
        std::free(raw);  // unchanged
        return;
    }
    g_swp.store(&s, std::memory_order_release);  // (never freed: see g_swp)
}

// ---- launchers defined in the kernel translation units ---------------------
int32_t launch_embed_pe(const int64_t*, const float*, const float*, int, int, int, int, float*, const int64_t*,
                        uint8_t*, hipStream_t);
int32_t launch_layer_norm(const float*, const float*, const float*, int, int, float*, hipStream_t);
int32_t launch_linear(const float*, const float*, const float*, const float*, const float*,
                      const float*, int, int, int, int, float*, hipStream_t);
// force_f32: the exact-f32 MFMA attention (a model whose q/k/v bound is outside the split-f16 range)
int32_t launch_attention(const float*, const uint8_t*, int, int, int, int, float*, hipStream_t, bool force_f32 = false);
int32_t launch_duration(const float*, int, int, int, const float* const*, float*, hipStream_t,
                        const float* ln_g = nullptr, const float* ln_b = nullptr, float* enc_out = nullptr,
                        const float* const* wsplit = nullptr);
int32_t launch_duration_count(const float*, int, int, int, const float* const*, float*, hipStream_t, const float*,
                              const float*, float*, float, int32_t*, int32_t*, int32_t*, unsigned*, int32_t*, int32_t,
                              const float* const* wsplit = nullptr);
bool duration_count_fusable(int, int);
int32_t launch_lr_count(const void*, int, float, int, int, int32_t*, int32_t*, int32_t*, hipStream_t);
int32_t launch_lr_count_sync(const void*, int, float, int, int, int32_t*, int32_t*, int32_t*, unsigned*, int32_t*,
                             int32_t, hipStream_t);
int32_t launch_lr_expand(const float*, const int32_t*, int, int, int, int, float*, hipStream_t);
int32_t launch_conv(const float*, const float*, const float*, const float*, const float*,
                    const float*, int, int, bool, int, int, int, int, float*, hipStream_t);
int32_t launch_add_pe(const float*, const float*, int, int, int, float*, hipStream_t);
int32_t launch_embed_pe_scaled(const int64_t*, const float*, const float*, int, int, int, int, float, float*, hipStream_t);
int32_t launch_convT(const float*, const float*, const float*, int, int, int, int, int, int,
                     float*, hipStream_t);
int32_t launch_conv_general(const float*, const float*, const float*, const float*, const float*, const float*, int,
                            int, int, int, int, int, int, int, float*, hipStream_t);

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int32_t fail(int32_t code, const char* what) {
    set_error(what);
    return code;
}

int32_t hip_status(hipError_t e, const char* where) {
    set_error(std::string(where) + ": " + hipGetErrorString(e));
    return static_cast<int32_t>(e);
}

static constexpr int kRates[4] = {4, 4, 2, 2};  // tts_model.py:244
// Receptive field of one audio sample in mel frames, per side: input_conv 1,
// ConvT1 ~1 (two taps), then ResBlock/ConvT stages at 4x..64x, 3 frames in
// total (tools/probe/receptive_field.py propagates the index intervals layer
// by layer).  A window widened by this many frames computes every sample of
// its centre exactly as the whole-utterance call does.
static constexpr int kVocHalo = 3;
// Longest regulated utterance the path accepts: 2^24 mel frames (2^30 audio
// samples, 13.5 h at 22.05 kHz); longer totals (a huge duration_scale or
// target durations) are M2_E_SHAPE, not a wrapped or truncated int32.
static constexpr int32_t kMaxFrames = 1 << 24;


// ---------------------------------------------------------------------------
// Weight table in M2TTSModel.state_dict() order (tts_model.py:303-343).
struct WSpec {
    std::string name;
    int64_t numel;
    bool is_int64;
};

static void add_layer(std::vector<WSpec>& t, const std::string& p, int64_t H) {
    t.push_back({p + ".self_attn.qkv.weight", 3 * H * H, false});
    t.push_back({p + ".self_attn.out_proj.weight", H * H, false});
    t.push_back({p + ".self_attn.out_proj.bias", H, false});
    t.push_back({p + ".ffn.linear1.weight", 2 * H * H, false});
    t.push_back({p + ".ffn.linear1.bias", 2 * H, false});
    t.push_back({p + ".ffn.linear2.weight", 2 * H * H, false});
    t.push_back({p + ".ffn.linear2.bias", H, false});
    t.push_back({p + ".norm1.weight", H, false});
    t.push_back({p + ".norm1.bias", H, false});
    t.push_back({p + ".norm2.weight", H, false});
    t.push_back({p + ".norm2.bias", H, false});
}

static std::vector<WSpec> weight_table(const m2_config& c) {
    std::vector<WSpec> t;
    const int64_t H = c.hidden_dim, M = c.mel_channels, C = c.vocoder_channels;
    t.push_back({"text_encoder.embedding.weight", (int64_t)c.vocab_size * H, false});
    t.push_back({"text_encoder.pos_encoding.pe", (int64_t)c.max_positions * H, false});
    for (int i = 0; i < c.text_encoder_layers; ++i) add_layer(t, "text_encoder.layers." + std::to_string(i), H);
    t.push_back({"text_encoder.norm.weight", H, false});
    t.push_back({"text_encoder.norm.bias", H, false});
    for (int j = 0; j < 2; ++j) {
        const std::string p = "duration_predictor.predictor.conv_layers." + std::to_string(j);
        t.push_back({p + ".conv.weight", H * H * 3, false});
        t.push_back({p + ".conv.bias", H, false});
        t.push_back({p + ".norm.weight", H, false});
        t.push_back({p + ".norm.bias", H, false});
        t.push_back({p + ".norm.running_mean", H, false});
        t.push_back({p + ".norm.running_var", H, false});
        t.push_back({p + ".norm.num_batches_tracked", 1, true});
    }
    t.push_back({"duration_predictor.predictor.projection.weight", H, false});
    t.push_back({"duration_predictor.predictor.projection.bias", 1, false});
    for (int i = 0; i < c.decoder_layers; ++i) add_layer(t, "decoder.layers." + std::to_string(i), H);
    t.push_back({"decoder.norm.weight", H, false});
    t.push_back({"decoder.norm.bias", H, false});
    t.push_back({"decoder.mel_projection.weight", M * H, false});
    t.push_back({"decoder.mel_projection.bias", M, false});
    t.push_back({"vocoder.input_conv.weight", C * M * 3, false});
    t.push_back({"vocoder.input_conv.bias", C, false});
    int64_t ch = C;
    for (int k = 0; k < 4; ++k) {
        const std::string p = "vocoder.upsamples." + std::to_string(k);
        t.push_back({p + ".weight", ch * (ch / 2) * 2 * kRates[k], false});
        t.push_back({p + ".bias", ch / 2, false});
        ch /= 2;
    }
    ch = C;
    for (int k = 0; k < 4; ++k) {
        ch /= 2;
        const std::string p = "vocoder.resblocks." + std::to_string(k);
        t.push_back({p + ".conv1.weight", ch * ch * 3, false});
        t.push_back({p + ".conv1.bias", ch, false});
        t.push_back({p + ".conv2.weight", ch * ch * 3, false});
        t.push_back({p + ".conv2.bias", ch, false});
    }
    t.push_back({"vocoder.output_conv.weight", ch * 3, false});
    t.push_back({"vocoder.output_conv.bias", 1, false});
    return t;
}

static bool config_ok(const m2_config* c) {
    if (!c) return false;
    const bool pos = c->vocab_size > 0 && c->hidden_dim > 0 && c->mel_channels > 0 &&
                     c->text_encoder_layers >= 0 && c->decoder_layers >= 0 && c->num_heads > 0 &&
                     c->vocoder_channels >= 16 && c->max_positions > 0;
    return pos && c->hidden_dim % c->num_heads == 0 && c->vocoder_channels % 16 == 0;
}

}  // namespace m2

// ---------------------------------------------------------------------------
struct m2_layer_w {
    const float *qkv_w, *out_w, *out_b, *ff1_w, *ff1_b, *ff2_w, *ff2_b, *n1_w, *n1_b, *n2_w, *n2_b;
    // B-fragment packs for the fused layer kernels (transformer_fused.hip)
    const float *qkv_p = nullptr, *out_p = nullptr, *ff1_p = nullptr, *ff2_p = nullptr;
    // the layer's attention scores (log2 units, scale folded) may leave the
    // f16 range: its one-launch form keeps the softmax base in f32 (TflLayer)
    bool wide_scores = false;
};

struct m2_model {
    m2_config cfg{};
    float* buf = nullptr;
    std::vector<const float*> ptr;  // per weight-table entry (nullptr for int64 entries)
    std::vector<m2_layer_w> enc, dec;
    const float *emb = nullptr, *pe = nullptr, *enc_nw = nullptr, *enc_nb = nullptr;
    const float* dur[10] = {};  // w1,b1,alpha1,beta1, w2,b2,alpha2,beta2, proj_w, proj_b
    // the duration convs' split-f16 fragments, used on the inference path
    // (fused final LayerNorm) when the static range bound allows (dur_split)
    const float* dur_split_w[2] = {};
    bool dur_split = false;
    const float *dec_nw = nullptr, *dec_nb = nullptr, *mel_w = nullptr, *mel_b = nullptr;
    const float* mel_p = nullptr;  // packed mel projection (fused path)
    bool tfused = false;           // transformer layers on ln_gemm + attention + post_attn
    const float *vin_w = nullptr, *vin_b = nullptr, *vout_w = nullptr, *vout_b = nullptr;
    const float *up_w[4] = {}, *up_b[4] = {};
    const float *rb_w1[4] = {}, *rb_b1[4] = {}, *rb_w2[4] = {}, *rb_b2[4] = {};
    // fused vocoder: packed weights
    float* vbuf = nullptr;
    m2::VocW vw{};
    bool fused = false;
    // split-f16 vocoder (vocoder_x3.hip): packed hi/lo weights; preferred when supported
    void* xbuf = nullptr;
    m2::VocX vx{};
    bool x3 = false;
    void* tbuf = nullptr;  // pipelined tail pack (stage1: vx.tp / vx.tpb, stage2: vx.tp2 / vx.tp2b)
    bool tailp = false;
    void* mbuf = nullptr;  // pipelined stage1 mid pack (vx.mp / vx.mpb)
    bool midp = false;
    bool x3_packed = false;  // split-f16 packs exist (m2_vocoder_select can switch x3 on/off)
    // streamed vocoder (m2_vocoder_set_chunking): chunks of chunk_frames mel
    // frames, each computed over a window widened by kVocHalo frames per side
    int chunk_frames = 0;
    // split-f16 range: non-finite-audio flag (host-mapped, vx.rflag is its
    // device address), what a raised flag does (m2_set_range_policy), and the
    // exact-f32 attention for weights whose q/k/v bound leaves the f16 range
    int32_t* rflag_host = nullptr;
    // range policy 1 on the fused vocoders: two device flag words used by
    // alternate calls (rseq parity) - the split kernels raise the call's word,
    // the exact-f32 redo kernels run only when it is raised, and the next
    // call's head kernel zeroes it
    int* rflag_dev = nullptr;
    mutable unsigned rseq = 0;
    // policy 1 on the pipelined tails: the tail's in-launch local redo
    // instead of the guarded exact-f32 launch (vocoder_redo.h); device copy
    const m2::VocRedoW* redo_w = nullptr;
    int range_policy = 0;
    // one-launch transformer layers: work-queue counters and the launch
    // sequence whose parity picks their set (one stream per model)
    unsigned* tflq = nullptr;
    mutable unsigned tfl_seq = 0;
    // device-T path: the count kernel's ticket word (after the queue words in
    // tflq) and the host-mapped [seq, T] pair the back half's first launch
    // posts (m2_frames_wait)
    unsigned* cnt_ticket = nullptr;
    int32_t* fpost_host = nullptr;
    int32_t* fpost_dev = nullptr;
    mutable int32_t fpost_seq = 0;
    bool att_f32 = false;
    // measurement: per m2_vocoder call, an event pair around each fused kernel
    mutable std::vector<hipEvent_t> prof_begin, prof_end;  // [call][kernel]
    mutable int prof_calls = 0;
    uint32_t prof_mask = ~0u;  // which kernels get an event pair (m2_profile_select)
    int prof_stride = 1;       // record on every prof_stride-th call (m2_profile_stride)
    mutable long prof_seen = 0;
};

using namespace m2;

namespace {

int32_t mask_kernel_launch(const int64_t* lengths, int B, int S, uint8_t* mask, hipStream_t st);

__global__ void padding_mask_kernel(const int64_t* __restrict__ lengths, int B, int S,
                                    uint8_t* __restrict__ mask) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * S) return;
    const int b = i / S, s = i - b * S;
    mask[i] = (int64_t)s < lengths[b] ? 1 : 0;  // components.py:236-240
}

int32_t mask_kernel_launch(const int64_t* lengths, int B, int S, uint8_t* mask, hipStream_t st) {
    if (B * S == 0) return M2_OK;
    hipLaunchKernelGGL(padding_mask_kernel, dim3(cdiv(B * S, 256)), dim3(256), 0, st, lengths, B, S, mask);
    M2_LAUNCHED("padding_mask_kernel");
    return M2_OK;
}

// Transformer stack scratch: the residual stream x and the padding mask, then
// one region used either by the three-launch layers (qkv, att, hid) or by the
// one-launch layers (two TflBufs sets, ping-pong between layers).
struct TfBufs {
    float *x, *qkv, *att, *hid;
    uint8_t* mask;
    TflBufs tfl[2];
};

template <typename A>
void carve_tf(A& a, int B, int N, int H, int heads, TfBufs* out) {
    const size_t R = (size_t)B * N;
    float* x = a.template take<float>(R * H);
    uint8_t* mask = a.template take<uint8_t>(R);
    const size_t three = align_up(R * 3 * H * 4, 256) + align_up(R * H * 4, 256) + align_up(R * 2 * H * 4, 256);
    const size_t one = tfl_supported(H, heads) ? 2 * align_up(tfl_bytes(B, N, H, heads), 256) : 0;
    unsigned char* region = a.template take<unsigned char>(std::max(three, one));
    if (!out) return;
    *out = TfBufs{};
    out->x = x;
    out->mask = mask;
    if (!region) return;
    out->qkv = reinterpret_cast<float*>(region);
    out->att = reinterpret_cast<float*>(region + align_up(R * 3 * H * 4, 256));
    out->hid = reinterpret_cast<float*>(region + align_up(R * 3 * H * 4, 256) + align_up(R * H * 4, 256));
    if (one) {
        tfl_carve(region, B, N, H, heads, &out->tfl[0]);
        tfl_carve(region + align_up(tfl_bytes(B, N, H, heads), 256), B, N, H, heads, &out->tfl[1]);
    }
}

size_t vocoder_max_cl(const m2_config& c, int T) {
    size_t best = (size_t)c.vocoder_channels * T;
    size_t ch = c.vocoder_channels, L = T;
    for (int k = 0; k < 4; ++k) {
        ch /= 2;
        L *= kRates[k];
        best = std::max(best, ch * L);
    }
    return best;
}

template <typename A>
void carve_voc(A& a, const m2_config& c, int B, int T, float** bufs) {
    const size_t n = (size_t)B * vocoder_max_cl(c, T);
    for (int i = 0; i < 3; ++i) {
        float* p = a.template take<float>(n);
        if (bufs) bufs[i] = p;
    }
}

// Streamed vocoder scratch: the mel window [B, M, W] (or [B, W, M]), its
// audio [B, 64 W] and the vocoder intermediates of a W-frame call, W = the
// widest window (chunk + 2 halo frames, at most T).
struct ChunkBufs {
    float *mel, *audio, *voc[3];
};

template <typename A>
void carve_chunked(A& a, const m2_config& c, int B, int T, int chunk, ChunkBufs* out) {
    const int W = std::min(T, chunk + 2 * kVocHalo);
    float* mel = a.template take<float>((size_t)B * c.mel_channels * W);
    float* audio = a.template take<float>((size_t)B * 64 * W);
    float* voc[3];
    carve_voc(a, c, B, W, voc);
    if (out) *out = ChunkBufs{mel, audio, {voc[0], voc[1], voc[2]}};
}

// Vocoder scratch of a T-frame call on this model (streamed when chunking is
// set and T exceeds one chunk).
size_t vocoder_ws_bytes(const m2_model* m, int B, int T) {
    Sizer s;
    if (m->chunk_frames > 0 && T > m->chunk_frames) carve_chunked(s, m->cfg, B, T, m->chunk_frames, nullptr);
    else carve_voc(s, m->cfg, B, T, nullptr);
    return s.off;
}

// Stage hand-off of m2_inference_front -> m2_inference_back: the encoder
// output, durations, frame prefix sums / totals / maximum and the padding mask.
struct FrontBufs {
    float *enc, *dur;
    int32_t *cum, *tot, *tmax;
    uint8_t* mask;
};

template <typename A>
void carve_front(A& a, int B, int S, int H, FrontBufs* out) {
    float* enc = a.template take<float>((size_t)B * S * H);
    float* dur = a.template take<float>((size_t)B * S);
    int32_t* cum = a.template take<int32_t>((size_t)B * (S + 1));
    int32_t* tot = a.template take<int32_t>((size_t)B);
    int32_t* tmax = a.template take<int32_t>(1);
    uint8_t* mask = a.template take<uint8_t>((size_t)B * S);
    if (out) *out = FrontBufs{enc, dur, cum, tot, tmax, mask};
}

// One pre-LN transformer layer (components.py:131-140), x updated in place;
// for the first decoder layer the residual source is the caller's input.
int32_t run_layer(const m2_model* m, const m2_layer_w& L, const float* x_in, float* x, TfBufs& wb,
                  const uint8_t* mask, int B, int N, hipStream_t st) {
    const int H = m->cfg.hidden_dim, R = B * N;
    int32_t rc;
    if (m->tfused) {
        if ((rc = launch_ln_gemm(x_in, L.n1_w, L.n1_b, L.qkv_p, nullptr, ACT_NONE, R, H, 3 * H, wb.qkv, st))) return rc;
        if ((rc = launch_attention(wb.qkv, mask, B, N, H, m->cfg.num_heads, wb.att, st, m->att_f32))) return rc;
        return launch_post_attn(wb.att, x_in, L.out_p, L.out_b, L.n2_w, L.n2_b, L.ff1_p, L.ff1_b, L.ff2_p, L.ff2_b, R, H,
                                x, st);
    }
    if ((rc = launch_linear(x_in, L.n1_w, L.n1_b, L.qkv_w, nullptr, nullptr, ACT_NONE, R, H, 3 * H, wb.qkv, st))) return rc;
    if ((rc = launch_attention(wb.qkv, mask, B, N, H, m->cfg.num_heads, wb.att, st, m->att_f32))) return rc;
    if ((rc = launch_linear(wb.att, nullptr, nullptr, L.out_w, L.out_b, x_in, ACT_NONE, R, H, H, x, st))) return rc;
    if ((rc = launch_linear(x, L.n2_w, L.n2_b, L.ff1_w, L.ff1_b, nullptr, ACT_RELU, R, H, 2 * H, wb.hid, st))) return rc;
    if ((rc = launch_linear(wb.hid, nullptr, nullptr, L.ff2_w, L.ff2_b, x, ACT_NONE, R, 2 * H, H, x, st))) return rc;
    return M2_OK;
}

// A stack of layers; x_in -> x (x_in may be x).  On the fused path each
// layer's post-attention kernel also runs the next layer's LN1 -> QKV on its
// row tile (and, with fin_W, the final LN -> projection into fin_out: then
// *fin_done), one launch per layer fewer; results are identical to the
// separate launches (same fp32 y into the same LayerNorm / GEMM code).
bool tf_chain(const m2_model* m) {
    const int H = m->cfg.hidden_dim;  // M2_TF_CHAIN=0: separate ln_gemm launches (A/B)
    return sw().tf_chain && m->tfused && tf_post_next_supported(H, 3 * H);
}

// The first layer's input rows built by its LN1 -> QKV launch (embedding /
// frame expansion fused in; tf_chain stacks only).
bool tf_first_fused(const m2_model* m, const std::vector<m2_layer_w>& layers) {
    return tf_chain(m) && !layers.empty() && tf_src_fused_supported(m->cfg.hidden_dim, 3 * m->cfg.hidden_dim);
}

// The next launch's work queue (its parity alternates the counter sets).
TflQueue tfl_queue(const m2_model* m) { return TflQueue{m->tflq, m->tfl_seq++}; }
// A launch that failed may not have zeroed the next counter set: restart both.
int32_t tfl_reset(const m2_model* m, hipStream_t st, int32_t rc) {
    (void)hipMemsetAsync(m->tflq, 0, kTflQueueWords * sizeof(unsigned), st);
    m->tfl_seq = 0;
    return rc;
}

// One-launch layers (transformer_layer.hip) for a stack of this model:
// heads == 2, H in {32, 64, 96}, the split-f16 transformer path.
// M2_TF_LAYER=0 keeps the three-launch layers (A/B comparisons, tests).
bool tfl_use(const m2_model* m, const std::vector<m2_layer_w>& layers) {
    return sw().tf_layer && m->tfused && !m->att_f32 && !layers.empty() &&
           tfl_supported(m->cfg.hidden_dim, m->cfg.num_heads);
}

// The layers of a stack whose first LN1 -> QKV (launch_tfl_first) already
// wrote wb.tfl[0]; x0 = layer 0's input rows (residual), x = the output
// stream.  The last layer also runs the final LN -> projection into fin_out
// when its width has an instantiation (*fin_done).
int32_t run_tfl(const m2_model* m, const std::vector<m2_layer_w>& layers, const float* x0, float* x, TfBufs& wb,
                const int64_t* lengths, int B, int N, hipStream_t st, const float* fin_g = nullptr,
                const float* fin_b = nullptr, const float* fin_W = nullptr, const float* fin_bias = nullptr,
                int fin_N = 0, float* fin_out = nullptr, bool* fin_done = nullptr, const int32_t* dN = nullptr) {
    const int H = m->cfg.hidden_dim, heads = m->cfg.num_heads, n = (int)layers.size();
    if (fin_done) *fin_done = false;
    const float* cur = x0;
    for (int l = 0; l < n; ++l) {
        const m2_layer_w& L = layers[l];
        TflLayer w{L.out_p, L.out_b, L.n2_w, L.n2_b, L.ff1_p, L.ff1_b, L.ff2_p, L.ff2_b};
        w.wide_scores = L.wide_scores;
        int next = 0, NN = 0;
        float* z = nullptr;
        if (l + 1 < n) {
            next = 1;
            w.gn = layers[l + 1].n1_w;
            w.bn = layers[l + 1].n1_b;
            w.Wn = layers[l + 1].qkv_p;
        } else if (fin_W && tfl_proj_supported(H, fin_N)) {
            next = 2;
            w.gn = fin_g;
            w.bn = fin_b;
            w.Wn = fin_W;
            w.bn2 = fin_bias;
            NN = fin_N;
            z = fin_out;
        }
        const int32_t rc = launch_tfl_layer(w, B, N, H, heads, lengths != nullptr, lengths, cur, x, wb.tfl[l & 1], next,
                                            wb.tfl[(l + 1) & 1], NN, z, tfl_queue(m), st, dN);
        if (rc) return tfl_reset(m, st, rc);
        if (next == 2 && fin_done) *fin_done = true;
        cur = x;
    }
    return M2_OK;
}

int32_t run_stack(const m2_model* m, const std::vector<m2_layer_w>& layers, const float* x_in, float* x, TfBufs& wb,
                  const uint8_t* mask, int B, int N, hipStream_t st, const float* fin_g = nullptr,
                  const float* fin_b = nullptr, const float* fin_W = nullptr, const float* fin_bias = nullptr,
                  int fin_N = 0, float* fin_out = nullptr, bool* fin_done = nullptr, bool qkv_ready = false) {
    const int H = m->cfg.hidden_dim, R = B * N, n = (int)layers.size();
    if (fin_done) *fin_done = false;
    int32_t rc;
    const bool chain = tf_chain(m);
    if (!chain) {
        const float* cur = x_in;
        for (const auto& L : layers) {
            if ((rc = run_layer(m, L, cur, x, wb, mask, B, N, st))) return rc;
            cur = x;
        }
        return M2_OK;
    }
    if (n == 0) return M2_OK;
    const float* cur = x_in;
    if (!qkv_ready && (rc = launch_ln_gemm(cur, layers[0].n1_w, layers[0].n1_b, layers[0].qkv_p, nullptr, ACT_NONE, R,
                                           H, 3 * H, wb.qkv, st)))
        return rc;
    for (int l = 0; l < n; ++l) {
        const m2_layer_w& L = layers[l];
        if ((rc = launch_attention(wb.qkv, mask, B, N, H, m->cfg.num_heads, wb.att, st, m->att_f32))) return rc;
        if (l + 1 < n) {
            const m2_layer_w& Nx = layers[l + 1];
            rc = launch_post_attn_next(wb.att, cur, L.out_p, L.out_b, L.n2_w, L.n2_b, L.ff1_p, L.ff1_b, L.ff2_p,
                                       L.ff2_b, R, H, x, Nx.n1_w, Nx.n1_b, Nx.qkv_p, nullptr, 3 * H, wb.qkv, st);
        } else if (fin_W && tf_post_next_supported(H, fin_N)) {
            rc = launch_post_attn_next(wb.att, cur, L.out_p, L.out_b, L.n2_w, L.n2_b, L.ff1_p, L.ff1_b, L.ff2_p,
                                       L.ff2_b, R, H, x, fin_g, fin_b, fin_W, fin_bias, fin_N, fin_out, st);
            if (!rc && fin_done) *fin_done = true;
        } else {
            rc = launch_post_attn(wb.att, cur, L.out_p, L.out_b, L.n2_w, L.n2_b, L.ff1_p, L.ff1_b, L.ff2_p, L.ff2_b, R,
                                  H, x, st);
        }
        if (rc) return rc;
        cur = x;
    }
    return M2_OK;
}

}  // namespace

extern "C" {

int32_t m2_abi_version(void) { return M2_ABI_VERSION; }

const char* m2_last_error(void) { return g_last_error.c_str(); }

int32_t m2_weight_count(const m2_config* cfg) {
    if (!config_ok(cfg)) return fail(M2_E_ARG, "m2_weight_count: invalid config");
    return (int32_t)weight_table(*cfg).size();
}

int32_t m2_weight_name(const m2_config* cfg, int32_t index, char* buf, int32_t buflen) {
    if (!config_ok(cfg) || !buf || buflen <= 0) return fail(M2_E_ARG, "m2_weight_name: bad argument");
    const auto t = weight_table(*cfg);
    if (index < 0 || index >= (int32_t)t.size()) return fail(M2_E_ARG, "m2_weight_name: index out of range");
    const std::string& n = t[index].name;
    if ((int32_t)n.size() + 1 > buflen) return fail(M2_E_ARG, "m2_weight_name: buffer too small");
    std::memcpy(buf, n.c_str(), n.size() + 1);
    return M2_OK;
}

int64_t m2_weight_numel(const m2_config* cfg, int32_t index) {
    if (!config_ok(cfg)) return fail(M2_E_ARG, "m2_weight_numel: invalid config");
    const auto t = weight_table(*cfg);
    if (index < 0 || index >= (int32_t)t.size()) return fail(M2_E_ARG, "m2_weight_numel: index out of range");
    return t[index].numel;
}

void m2_reload_switches(void) { reload_switches(); }

int32_t m2_model_create(const m2_config* cfg, const void* const* weights, int32_t n_weights,
                        void* stream, m2_model** out) {
    reload_switches();  // the developer switches of this handle's creation (m2_common.h)
    M2_CHECK_ARG(config_ok(cfg), "m2_model_create: invalid config");
    M2_CHECK_ARG(weights && out, "m2_model_create: null argument");
    const auto table = weight_table(*cfg);
    if (n_weights != (int32_t)table.size()) return fail(M2_E_WEIGHTS, "m2_model_create: weight count mismatch");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int H = cfg->hidden_dim;

    // Layout: every fp32 weight copied verbatim, then 2x(alpha,beta) for the
    // BatchNorm inference form; 64-float aligned carves.
    std::vector<size_t> off(table.size(), 0);
    size_t total = 0;
    for (size_t i = 0; i < table.size(); ++i) {
        if (table[i].is_int64) continue;
        total = align_up(total, 64);
        off[i] = total;
        total += (size_t)table[i].numel;
        M2_CHECK_ARG(weights[i] != nullptr, "m2_model_create: null weight pointer");
    }
    total = align_up(total, 64);
    const size_t bn_off = total;
    total += 4 * (size_t)H;
    total = align_up(total, 64);
    const size_t dw_off = total;  // duration conv weights, B-fragment order, 2 layers
    total += 2 * 3 * (size_t)H * H;
    total = align_up(total, 64);
    const size_t dws_off = total;  // the same as split-f16 hi/lo fragments (pack_bfrag_split)
    total += 2 * 3 * (size_t)H * H;
    total = align_up(total, 64);
    const size_t tf_off = total;  // fused-layer B-fragment packs: 8H^2 per layer + mel projection
    const int n_layers = cfg->text_encoder_layers + cfg->decoder_layers;
    total += (size_t)n_layers * 8 * H * H + (size_t)cfg->mel_channels * H;

    auto* m = new m2_model();
    m->cfg = *cfg;
    hipError_t e = hipMalloc(&m->buf, total * sizeof(float));
    if (e != hipSuccess) { delete m; return hip_status(e, "hipMalloc(model)"); }
    auto bail = [&](hipError_t err, const char* w) { (void)hipFree(m->buf); delete m; return hip_status(err, w); };
    for (size_t i = 0; i < table.size(); ++i) {
        if (table[i].is_int64) continue;
        e = hipMemcpyAsync(m->buf + off[i], weights[i], table[i].numel * sizeof(float), hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return bail(e, "hipMemcpyAsync(weight)");
    }

    // name -> index
    auto idx = [&](const std::string& n) {
        for (size_t i = 0; i < table.size(); ++i) if (table[i].name == n) return (int)i;
        return -1;
    };
    m->ptr.resize(table.size(), nullptr);
    for (size_t i = 0; i < table.size(); ++i) if (!table[i].is_int64) m->ptr[i] = m->buf + off[i];
    auto P = [&](const std::string& n) { return m->ptr[idx(n)]; };

    // BatchNorm1d eval: alpha = gamma / sqrt(var + eps), beta' = beta - mean * alpha
    // (ATen batch_norm_cpu_collect_linear_and_constant_terms, fp32).
    std::vector<float> host(4 * (size_t)H), bnw(H), bnb(H), bnm(H), bnv(H);
    for (int j = 0; j < 2; ++j) {
        const std::string p = "duration_predictor.predictor.conv_layers." + std::to_string(j) + ".norm.";
        const float* src[4] = {static_cast<const float*>(weights[idx(p + "weight")]), static_cast<const float*>(weights[idx(p + "bias")]),
                               static_cast<const float*>(weights[idx(p + "running_mean")]), static_cast<const float*>(weights[idx(p + "running_var")])};
        float* dst[4] = {bnw.data(), bnb.data(), bnm.data(), bnv.data()};
        for (int q = 0; q < 4; ++q) {
            e = hipMemcpyAsync(dst[q], src[q], H * sizeof(float), hipMemcpyDeviceToHost, st);
            if (e != hipSuccess) return bail(e, "hipMemcpyAsync(bn)");
        }
        e = hipStreamSynchronize(st);
        if (e != hipSuccess) return bail(e, "hipStreamSynchronize");
        for (int c = 0; c < H; ++c) {
            const float invstd = 1.0f / std::sqrt(bnv[c] + 1e-5f);
            const float a = invstd * bnw[c];
            host[(2 * j) * H + c] = a;
            host[(2 * j + 1) * H + c] = bnb[c] - bnm[c] * a;
        }
    }
    // Duration convs: W[co][ci][tap] -> GEMM B matrix [co][tap*H + ci] -> B-fragment order
    // (exact-f32 MFMA) and split-f16 hi/lo fragments (v_mfma_f32_16x16x32_f16).
    std::vector<float> dpack(2 * 3 * (size_t)H * H), dspack(2 * 3 * (size_t)H * H);
    bool dsplit = true;
    double dconv_rows[2] = {0.0, 0.0};  // max over co of sum_{ci, tap} |W[co][ci][tap]|
    std::vector<float> dconv_bias[2];
    for (int j = 0; j < 2; ++j) {
        const std::string n = "duration_predictor.predictor.conv_layers." + std::to_string(j) + ".conv.weight";
        std::vector<float> w((size_t)3 * H * H), wt((size_t)3 * H * H);
        e = hipMemcpyAsync(w.data(), weights[idx(n)], w.size() * sizeof(float), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return bail(e, "hipMemcpyAsync(duration conv)");
        for (int co = 0; co < H; ++co)
            for (int ci = 0; ci < H; ++ci)
                for (int k = 0; k < 3; ++k) wt[(size_t)co * 3 * H + k * H + ci] = w[((size_t)co * H + ci) * 3 + k];
        const std::vector<float> pk = pack_bfrag(wt.data(), H, 3 * H);
        std::copy(pk.begin(), pk.end(), dpack.begin() + (size_t)j * 3 * H * H);
        std::vector<float> pks;
        if (pack_bfrag_split(wt.data(), H, 3 * H, &pks)) std::copy(pks.begin(), pks.end(), dspack.begin() + (size_t)j * 3 * H * H);
        else dsplit = false;
        for (int co = 0; co < H; ++co) {
            double r = 0.0;
            for (int k = 0; k < 3 * H; ++k) r += std::fabs((double)wt[(size_t)co * 3 * H + k]);
            dconv_rows[j] = std::max(dconv_rows[j], r);
        }
        dconv_bias[j].resize(H);
        const std::string nb = "duration_predictor.predictor.conv_layers." + std::to_string(j) + ".conv.bias";
        e = hipMemcpyAsync(dconv_bias[j].data(), weights[idx(nb)], H * sizeof(float), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return bail(e, "hipMemcpyAsync(duration conv bias)");
    }
    e = hipMemcpyAsync(m->buf + dw_off, dpack.data(), dpack.size() * sizeof(float), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return bail(e, "hipMemcpyAsync(duration pack)");
    e = hipMemcpyAsync(m->buf + dws_off, dspack.data(), dspack.size() * sizeof(float), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return bail(e, "hipMemcpyAsync(duration split pack)");
    // Split-f16 range of the duration convs on the inference path, where their
    // input is the encoder's final LayerNorm (|LN| <= sqrt(H-1) max|gamma| +
    // max|beta|) and conv2's input is BN(conv1) after ReLU (<= max|alpha| (row
    // sum |W1| x that + max|b1|) + max|beta'|): checked once here against half
    // the f16 range, as the transformer's bound below; outside it (or with a
    // weight outside the f16 range) the exact-f32 MFMA convs stay.
    {
        std::vector<float> g(H), bb(H);
        e = hipMemcpyAsync(g.data(), weights[idx("text_encoder.norm.weight")], H * sizeof(float), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess)
            e = hipMemcpyAsync(bb.data(), weights[idx("text_encoder.norm.bias")], H * sizeof(float), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return bail(e, "hipMemcpyAsync(encoder norm)");
        double ga = 0.0, ba = 0.0, b1a = 0.0, a1a = 0.0, c1a = 0.0;
        for (int c = 0; c < H; ++c) {
            ga = std::max(ga, (double)std::fabs(g[c]));
            ba = std::max(ba, (double)std::fabs(bb[c]));
            b1a = std::max(b1a, (double)std::fabs(dconv_bias[0][c]));
            a1a = std::max(a1a, (double)std::fabs(host[c]));
            c1a = std::max(c1a, (double)std::fabs(host[H + c]));
        }
        const double x0 = std::sqrt((double)std::max(H - 1, 1)) * ga + ba;
        const double x1 = a1a * (dconv_rows[0] * x0 + b1a) + c1a;
        m->dur_split = dsplit && x0 < 32768.0 && x1 < 32768.0;
    }
    e = hipMemcpyAsync(m->buf + bn_off, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return bail(e, "hipMemcpyAsync(bn up)");
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return bail(e, "hipStreamSynchronize");

    m->emb = P("text_encoder.embedding.weight");
    m->pe = P("text_encoder.pos_encoding.pe");
    auto layer = [&](const std::string& p) {
        return m2_layer_w{P(p + ".self_attn.qkv.weight"), P(p + ".self_attn.out_proj.weight"), P(p + ".self_attn.out_proj.bias"),
                          P(p + ".ffn.linear1.weight"), P(p + ".ffn.linear1.bias"), P(p + ".ffn.linear2.weight"),
                          P(p + ".ffn.linear2.bias"), P(p + ".norm1.weight"), P(p + ".norm1.bias"),
                          P(p + ".norm2.weight"), P(p + ".norm2.bias")};
    };
    for (int i = 0; i < cfg->text_encoder_layers; ++i) m->enc.push_back(layer("text_encoder.layers." + std::to_string(i)));
    for (int i = 0; i < cfg->decoder_layers; ++i) m->dec.push_back(layer("decoder.layers." + std::to_string(i)));
    // Fused transformer layers: pack qkv / out / ffn / mel-projection weights
    // in B-fragment order (M2_TF_UNFUSED=1 keeps the five-linear layer).
    m->tfused = tf_fused_supported(H, 3 * H) && tf_fused_supported(H, cfg->mel_channels) &&
                !sw().tf_unfused;
    if (m->tfused) {
        size_t o = tf_off;
        auto pack_up = [&](const std::string& n, int N, int K, const float** slot) -> hipError_t {
            std::vector<float> w((size_t)N * K);
            hipError_t er = hipMemcpyAsync(w.data(), weights[idx(n)], w.size() * sizeof(float), hipMemcpyDeviceToHost, st);
            if (er == hipSuccess) er = hipStreamSynchronize(st);
            if (er != hipSuccess) return er;
            std::vector<float> pk;
            if (!pack_bfrag_split(w.data(), N, K, &pk)) return hipErrorInvalidValue;  // |w| >= 65504
            er = hipMemcpyAsync(m->buf + o, pk.data(), pk.size() * sizeof(float), hipMemcpyHostToDevice, st);
            if (er == hipSuccess) er = hipStreamSynchronize(st);
            *slot = m->buf + o;
            o += pk.size();
            return er;
        };
        for (int i = 0; i < n_layers && e == hipSuccess; ++i) {
            const bool is_enc = i < cfg->text_encoder_layers;
            m2_layer_w& L = is_enc ? m->enc[i] : m->dec[i - cfg->text_encoder_layers];
            const std::string p = (is_enc ? "text_encoder.layers." + std::to_string(i)
                                          : "decoder.layers." + std::to_string(i - cfg->text_encoder_layers));
            if (e == hipSuccess) e = pack_up(p + ".self_attn.qkv.weight", 3 * H, H, &L.qkv_p);
            if (e == hipSuccess) e = pack_up(p + ".self_attn.out_proj.weight", H, H, &L.out_p);
            if (e == hipSuccess) e = pack_up(p + ".ffn.linear1.weight", 2 * H, H, &L.ff1_p);
            if (e == hipSuccess) e = pack_up(p + ".ffn.linear2.weight", H, 2 * H, &L.ff2_p);
        }
        if (e == hipSuccess) e = pack_up("decoder.mel_projection.weight", cfg->mel_channels, H, &m->mel_p);
        if (e == hipErrorInvalidValue) {  // a weight outside the f16 range: keep the fp32 five-linear layers
            m->tfused = false;
            e = hipSuccess;
        }
        if (e != hipSuccess) return bail(e, "pack transformer weights");
    }
    // Split-f16 range of the transformer.  Its split operands are LayerNorm
    // outputs (|x^| <= sqrt(H-1) for a normalised row, so |LN| <= sqrt(H-1)
    // max|gamma| + max|beta|), q/k/v = W_qkv LN1 (<= max row sum |W| x that),
    // attention outputs (convex combinations of v) and ReLU(FFN1(LN2)) - all
    // bounded by the weights, so the check is made once, here: past half the
    // f16 range the layers use the fp32 linears and the exact-f32 attention.
    {
        double worst = 0.0;
        auto host = [&](const std::string& n) {
            const int i = idx(n);
            std::vector<float> h((size_t)table[i].numel);
            hipError_t er = hipMemcpyAsync(h.data(), weights[i], h.size() * sizeof(float), hipMemcpyDeviceToHost, st);
            if (er == hipSuccess) er = hipStreamSynchronize(st);
            if (er != hipSuccess) h.assign(h.size(), INFINITY);
            return h;
        };
        auto amax = [](const std::vector<float>& v) {
            double a = 0.0;
            for (float x : v) a = std::max(a, (double)std::fabs(x));
            return a;
        };
        auto ln_bound = [&](const std::string& p) {
            return std::sqrt((double)std::max(H - 1, 1)) * amax(host(p + ".weight")) + amax(host(p + ".bias"));
        };
        auto row_sum = [&](const std::string& n, int N, int K) {
            const std::vector<float> w = host(n);
            double best = 0.0;
            for (int r = 0; r < N; ++r) {
                double s = 0.0;
                for (int k = 0; k < K; ++k) s += std::fabs(w[(size_t)r * K + k]);
                best = std::max(best, s);
            }
            return best;
        };
        // scores in log2 units, |q.k| scale log2(e) <= sum over a head's dims of
        // |q_d| |k_d| (each bounded by its row sum of |W_qkv| x the LN1 bound)
        // x scale log2(e): the head_dim-48 wave-specialised attention holds its
        // softmax base m (<= the largest score) as an f16 hi / lo pair, finite
        // while |m| < 65520, so a layer whose bound reaches the f16 maximum
        // runs the f32-base form (m2_layer_w::wide_scores; the seeded stage2
        // weights bound at ~3.5e4)
        const int heads = cfg->num_heads, hd = H / std::max(heads, 1);
        const double sl2 = 1.0 / std::sqrt((double)hd) * 1.4426950408889634;
        for (int i = 0; i < n_layers; ++i) {
            const bool is_enc = i < cfg->text_encoder_layers;
            const std::string p = is_enc ? "text_encoder.layers." + std::to_string(i)
                                         : "decoder.layers." + std::to_string(i - cfg->text_encoder_layers);
            const double b1 = ln_bound(p + ".norm1"), b2 = ln_bound(p + ".norm2");
            const double qkv = row_sum(p + ".self_attn.qkv.weight", 3 * H, H) * b1;
            {
                // rows of W_qkv: the reference's reshape (3, heads, head_dim)
                const std::vector<float> w = host(p + ".self_attn.qkv.weight");
                auto rs = [&](int r) {
                    double a = 0.0;
                    for (int k = 0; k < H; ++k) a += std::fabs(w[(size_t)r * H + k]);
                    return a * b1;
                };
                double sb = 0.0;
                for (int h = 0; h < heads; ++h) {
                    double acc = 0.0;
                    for (int d = 0; d < hd; ++d) acc += rs(h * hd + d) * rs(H + h * hd + d);
                    sb = std::max(sb, acc * sl2);
                }
                m2_layer_w& L = is_enc ? m->enc[i] : m->dec[i - cfg->text_encoder_layers];
                L.wide_scores = !(sb < 65504.0);
            }
            const double hid = row_sum(p + ".ffn.linear1.weight", 2 * H, H) * b2 + amax(host(p + ".ffn.linear1.bias"));
            worst = std::max(worst, std::max(std::max(b1, b2), std::max(qkv, hid)));
        }
        if (cfg->decoder_layers > 0) worst = std::max(worst, ln_bound("decoder.norm"));
        if (!(worst < 32768.0)) {
            m->tfused = false;
            m->att_f32 = true;
        }
    }
    m->enc_nw = P("text_encoder.norm.weight");
    m->enc_nb = P("text_encoder.norm.bias");
    for (int j = 0; j < 2; ++j) {
        const std::string p = "duration_predictor.predictor.conv_layers." + std::to_string(j) + ".conv.";
        m->dur[4 * j + 0] = m->buf + dw_off + (size_t)j * 3 * H * H;
        m->dur[4 * j + 1] = P(p + "bias");
        m->dur[4 * j + 2] = m->buf + bn_off + (2 * j) * H;
        m->dur[4 * j + 3] = m->buf + bn_off + (2 * j + 1) * H;
    }
    m->dur_split_w[0] = m->buf + dws_off;
    m->dur_split_w[1] = m->buf + dws_off + (size_t)3 * H * H;
    m->dur[8] = P("duration_predictor.predictor.projection.weight");
    m->dur[9] = P("duration_predictor.predictor.projection.bias");
    m->dec_nw = P("decoder.norm.weight");
    m->dec_nb = P("decoder.norm.bias");
    m->mel_w = P("decoder.mel_projection.weight");
    m->mel_b = P("decoder.mel_projection.bias");
    m->vin_w = P("vocoder.input_conv.weight");
    m->vin_b = P("vocoder.input_conv.bias");
    for (int k = 0; k < 4; ++k) {
        const std::string u = "vocoder.upsamples." + std::to_string(k);
        const std::string r = "vocoder.resblocks." + std::to_string(k);
        m->up_w[k] = P(u + ".weight");
        m->up_b[k] = P(u + ".bias");
        m->rb_w1[k] = P(r + ".conv1.weight");
        m->rb_b1[k] = P(r + ".conv1.bias");
        m->rb_w2[k] = P(r + ".conv2.weight");
        m->rb_b2[k] = P(r + ".conv2.bias");
    }
    m->vout_w = P("vocoder.output_conv.weight");
    m->vout_b = P("vocoder.output_conv.bias");

    // Fused vocoder: pack conv / convT weights into MFMA A-fragment order.
    m->fused = vocoder_fused_supported(cfg->mel_channels, cfg->vocoder_channels) && !sw().voc_perlayer;
    if (m->fused) {
        auto fetch = [&](const std::string& n) {
            const int i = idx(n);
            std::vector<float> h((size_t)table[i].numel);
            hipError_t er = hipMemcpyAsync(h.data(), weights[i], h.size() * sizeof(float), hipMemcpyDeviceToHost, st);
            if (er == hipSuccess) er = hipStreamSynchronize(st);
            if (er != hipSuccess) h.clear();
            return h;
        };
        std::vector<std::vector<float>> parts;
        std::vector<const float**> slots;
        auto add = [&](std::vector<float> v, const float** slot) { parts.push_back(std::move(v)); slots.push_back(slot); };
        const int M = cfg->mel_channels, C = cfg->vocoder_channels;
        auto wi = fetch("vocoder.input_conv.weight");
        if (wi.empty()) return bail(hipErrorUnknown, "fetch vocoder weights");
        add(pack_conv3(wi.data(), C, M), &m->vw.wi);
        add(fetch("vocoder.input_conv.bias"), &m->vw.bi);
        int ch = C;
        for (int k = 0; k < 4; ++k) {
            const std::string u = "vocoder.upsamples." + std::to_string(k);
            const std::string r = "vocoder.resblocks." + std::to_string(k);
            auto wt = fetch(u + ".weight");
            add(pack_convT(wt.data(), ch, ch / 2, kRates[k]), &m->vw.wt[k]);
            add(fetch(u + ".bias"), &m->vw.bt[k]);
            ch /= 2;
            auto w1 = fetch(r + ".conv1.weight");
            add(pack_conv3(w1.data(), ch, ch), &m->vw.w1[k]);
            add(fetch(r + ".conv1.bias"), &m->vw.b1[k]);
            auto w2 = fetch(r + ".conv2.weight");
            add(pack_conv3(w2.data(), ch, ch), &m->vw.w2[k]);
            add(fetch(r + ".conv2.bias"), &m->vw.b2[k]);
            if (k == 3 && ch == 8 && kRates[3] == 2) {  // the two-phase forms of the last stage
                add(pack_convT2_paired(wt.data(), 2 * ch), &m->vw.wt4p);
                add(pack_conv3_2p(w1.data()), &m->vw.w1p);
                add(pack_conv3_2p(w2.data()), &m->vw.w2p);
            }
        }
        if ((M == 64 && C == 128) || (M == 80 && C == 256)) {  // the exact-f32 head's composed input conv o ConvT1
            std::vector<uint16_t> hw_unused;
            std::vector<float> hb, he;
            bool hok = true;
            const auto bi = fetch("vocoder.input_conv.bias"), wt0 = fetch("vocoder.upsamples.0.weight"),
                       bt0 = fetch("vocoder.upsamples.0.bias");
            if (pack_x3_head_comp(wi.data(), bi.data(), wt0.data(), bt0.data(), M, M, C, &hw_unused, &hb, &he, &hok)) {
                add(pack_f32_head_comp(wi.data(), wt0.data(), M, C), &m->vw.hcw);
                add(std::move(hb), &m->vw.hcb);
                add(std::move(he), &m->vw.hce);
            }
        }
        size_t tot = 0;
        std::vector<size_t> offs;
        for (auto& v : parts) { tot = align_up(tot, 64); offs.push_back(tot); tot += v.size(); }
        std::vector<float> host(tot, 0.f);
        for (size_t i = 0; i < parts.size(); ++i) std::copy(parts[i].begin(), parts[i].end(), host.begin() + offs[i]);
        e = hipMalloc(&m->vbuf, std::max<size_t>(tot, 1) * sizeof(float));
        if (e != hipSuccess) return bail(e, "hipMalloc(vocoder pack)");
        e = hipMemcpyAsync(m->vbuf, host.data(), tot * sizeof(float), hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) { (void)hipFree(m->vbuf); return bail(e, "upload vocoder pack"); }
        for (size_t i = 0; i < parts.size(); ++i) *slots[i] = m->vbuf + offs[i];
        m->vw.wo = m->vout_w;
        m->vw.bo = m->vout_b;

        // Split-f16 packs (default path when the shapes are supported and every
        // weight is inside the f16 range; M2_VOC_F32=1 keeps the exact-f32 MFMA).
        if (vocoder_x3_supported(M, C) && !sw().voc_f32) {
            bool ok = true;
            std::vector<std::vector<uint16_t>> xp;
            std::vector<const vx_u32x4**> xs;
            xp.push_back(pack_x3_conv3(wi.data(), C, M, vocoder_x3_mel_pad(M), &ok, false));
            xs.push_back(&m->vx.wi);
            int c2 = C;
            for (int k = 0; k < 4; ++k) {
                const std::string u = "vocoder.upsamples." + std::to_string(k);
                const std::string r = "vocoder.resblocks." + std::to_string(k);
                auto wt = fetch(u + ".weight");
                xp.push_back(pack_x3_convT(wt.data(), c2, c2 / 2, kRates[k], &ok));
                xs.push_back(&m->vx.wt[k]);
                c2 /= 2;
                auto w1 = fetch(r + ".conv1.weight");
                xp.push_back(pack_x3_conv3(w1.data(), c2, c2, c2, &ok, false));
                xs.push_back(&m->vx.w1[k]);
                auto w2 = fetch(r + ".conv2.weight");
                xp.push_back(pack_x3_conv3(w2.data(), c2, c2, c2, &ok, true));
                xs.push_back(&m->vx.w2[k]);
            }
            // stage1 head: input_conv composed into ConvT1 (fp32 bias / edge
            // tables ride in the same buffer as u16 pairs)
            const vx_u32x4* hcb_at = nullptr;
            const vx_u32x4* hce_at = nullptr;
            if ((M == 64 && C == 128) || (M == 80 && C == 256)) {
                std::vector<uint16_t> hw;
                std::vector<float> hb, he;
                const auto bi = fetch("vocoder.input_conv.bias"), wt0 = fetch("vocoder.upsamples.0.weight"),
                           bt0 = fetch("vocoder.upsamples.0.bias");
                bool hok = true;
                if (pack_x3_head_comp(wi.data(), bi.data(), wt0.data(), bt0.data(), M, vocoder_x3_mel_pad(M), C, &hw,
                                      &hb, &he, &hok) && hok) {
                    auto as_u16 = [](const std::vector<float>& f) {
                        std::vector<uint16_t> u(f.size() * 2);
                        std::memcpy(u.data(), f.data(), f.size() * sizeof(float));
                        return u;
                    };
                    xp.push_back(std::move(hw));
                    xs.push_back(&m->vx.hc);
                    xp.push_back(as_u16(hb));
                    xs.push_back(&hcb_at);
                    xp.push_back(as_u16(he));
                    xs.push_back(&hce_at);
                }
            }
            if (ok) {
                size_t xt = 0;
                std::vector<size_t> xo;
                for (auto& v : xp) { xt = align_up(xt, 128); xo.push_back(xt); xt += v.size(); }
                std::vector<uint16_t> hx(xt, 0);
                for (size_t i = 0; i < xp.size(); ++i) std::copy(xp[i].begin(), xp[i].end(), hx.begin() + xo[i]);
                e = hipMalloc(&m->xbuf, std::max<size_t>(xt, 1) * sizeof(uint16_t));
                if (e != hipSuccess) { (void)hipFree(m->vbuf); return bail(e, "hipMalloc(x3 pack)"); }
                e = hipMemcpyAsync(m->xbuf, hx.data(), xt * sizeof(uint16_t), hipMemcpyHostToDevice, st);
                if (e == hipSuccess) e = hipStreamSynchronize(st);
                if (e != hipSuccess) { (void)hipFree(m->vbuf); (void)hipFree(m->xbuf); return bail(e, "upload x3 pack"); }
                for (size_t i = 0; i < xp.size(); ++i)
                    *xs[i] = reinterpret_cast<const vx_u32x4*>(static_cast<uint16_t*>(m->xbuf) + xo[i]);
                m->vx.hcb = reinterpret_cast<const float*>(hcb_at);
                m->vx.hce = reinterpret_cast<const float*>(hce_at);
                m->vx.bi = m->vw.bi;
                for (int k = 0; k < 4; ++k) {
                    m->vx.bt[k] = m->vw.bt[k];
                    m->vx.b1[k] = m->vw.b1[k];
                    m->vx.b2[k] = m->vw.b2[k];
                }
                m->vx.wo = m->vw.wo;
                m->vx.bo = m->vw.bo;
                m->x3 = true;
                m->x3_packed = true;
                // stage1 / stage2: the last two upsampling stages as one
                // pipelined kernel (M2_VOC_TAIL_X3=1 keeps the x3 tail kernel).
                const bool s2tail = M == 80 && C == 256;
                if (((M == 64 && C == 128) || s2tail) && !sw().voc_tail_x3) {
                    const char* names[14] = {
                        "vocoder.upsamples.2.weight",         "vocoder.upsamples.2.bias",
                        "vocoder.resblocks.2.conv1.weight", "vocoder.resblocks.2.conv1.bias",
                        "vocoder.resblocks.2.conv2.weight", "vocoder.resblocks.2.conv2.bias",
                        "vocoder.upsamples.3.weight",         "vocoder.upsamples.3.bias",
                        "vocoder.resblocks.3.conv1.weight", "vocoder.resblocks.3.conv1.bias",
                        "vocoder.resblocks.3.conv2.weight", "vocoder.resblocks.3.conv2.bias",
                        "vocoder.output_conv.weight",         "vocoder.output_conv.bias"};
                    std::vector<float> hw[14];
                    bool got = true;
                    for (int i = 0; i < 14; ++i) got = got && !(hw[i] = fetch(names[i])).empty();
                    const TailpSrc src{hw[0].data(), hw[1].data(), hw[2].data(),  hw[3].data(),  hw[4].data(),
                                       hw[5].data(), hw[6].data(), hw[7].data(),  hw[8].data(),  hw[9].data(),
                                       hw[10].data(), hw[11].data(), hw[12].data(), hw[13].data()};
                    std::vector<uint16_t> pw;
                    std::vector<float> pb;
                    bool rok = true;
                    if (got && (s2tail ? pack_tailp2(src, &pw, &pb, &rok) : pack_tailp(src, &pw, &pb, &rok)) && rok) {
                        const size_t wb = pw.size() * sizeof(uint16_t);
                        e = hipMalloc(&m->tbuf, wb + pb.size() * sizeof(float));
                        if (e == hipSuccess) e = hipMemcpyAsync(m->tbuf, pw.data(), wb, hipMemcpyHostToDevice, st);
                        if (e == hipSuccess)
                            e = hipMemcpyAsync(static_cast<char*>(m->tbuf) + wb, pb.data(), pb.size() * sizeof(float),
                                               hipMemcpyHostToDevice, st);
                        if (e == hipSuccess) e = hipStreamSynchronize(st);
                        if (e != hipSuccess) {
                            (void)hipFree(m->vbuf);
                            (void)hipFree(m->xbuf);
                            if (m->tbuf) (void)hipFree(m->tbuf);
                            return bail(e, "upload tailp pack");
                        }
                        const auto* tw = static_cast<const vx_u32x4*>(m->tbuf);
                        const auto* tb = reinterpret_cast<const float*>(static_cast<char*>(m->tbuf) + wb);
                        if (s2tail) {
                            m->vx.tp2 = tw;
                            m->vx.tp2b = tb;
                        } else {
                            m->vx.tp = tw;
                            m->vx.tpb = tb;
                        }
                        m->tailp = true;
                    }
                }
                // stage1: the second upsampling stage as one pipelined kernel
                // (M2_VOC_MID_X3=1 keeps the x3 mid kernel).
                if (M == 64 && C == 128 && !sw().voc_mid_x3) {
                    const char* names[6] = {"vocoder.upsamples.1.weight",         "vocoder.upsamples.1.bias",
                                            "vocoder.resblocks.1.conv1.weight", "vocoder.resblocks.1.conv1.bias",
                                            "vocoder.resblocks.1.conv2.weight", "vocoder.resblocks.1.conv2.bias"};
                    std::vector<float> hw[6];
                    bool got = true;
                    for (int i = 0; i < 6; ++i) got = got && !(hw[i] = fetch(names[i])).empty();
                    const MidpSrc src{hw[0].data(), hw[1].data(), hw[2].data(), hw[3].data(), hw[4].data(), hw[5].data()};
                    std::vector<uint16_t> pw;
                    std::vector<float> pb;
                    bool rok = true;
                    if (got && pack_midp(src, &pw, &pb, &rok) && rok) {
                        const size_t wb = pw.size() * sizeof(uint16_t);
                        e = hipMalloc(&m->mbuf, wb + pb.size() * sizeof(float));
                        if (e == hipSuccess) e = hipMemcpyAsync(m->mbuf, pw.data(), wb, hipMemcpyHostToDevice, st);
                        if (e == hipSuccess)
                            e = hipMemcpyAsync(static_cast<char*>(m->mbuf) + wb, pb.data(), pb.size() * sizeof(float),
                                               hipMemcpyHostToDevice, st);
                        if (e == hipSuccess) e = hipStreamSynchronize(st);
                        if (e != hipSuccess) {
                            (void)hipFree(m->vbuf);
                            (void)hipFree(m->xbuf);
                            if (m->tbuf) (void)hipFree(m->tbuf);
                            if (m->mbuf) (void)hipFree(m->mbuf);
                            return bail(e, "upload midp pack");
                        }
                        m->vx.mp = static_cast<const vx_u32x4*>(m->mbuf);
                        m->vx.mpb = reinterpret_cast<const float*>(static_cast<char*>(m->mbuf) + wb);
                        m->midp = true;
                    }
                }
            }
        }
    }
    // the split path's non-finite-audio flag, host-mapped so the host can read
    // it without a copy (m2_model_check, the M2_E_RANGE check on entry)
    {
        void* h = nullptr;
        void* d = nullptr;
        e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            if (h) (void)hipHostFree(h);
            m2_model_destroy(m);
            return hip_status(e, "hipHostMalloc(range flag)");
        }
        std::memset(h, 0, 64);
        m->rflag_host = static_cast<int32_t*>(h);
        m->vx.rflag = static_cast<int*>(d);
        void* dv = nullptr;
        e = hipMalloc(&dv, 64);
        if (e == hipSuccess) e = hipMemsetAsync(dv, 0, 64, st);
        if (e != hipSuccess) {
            if (dv) (void)hipFree(dv);
            m2_model_destroy(m);
            return hip_status(e, "hipMalloc(range flags)");
        }
        m->rflag_dev = static_cast<int*>(dv);
    }
    // the local redo's weight table (range policy "fallback" on the pipelined
    // tails, vocoder_redo.h): the raw fp32 vocoder weights, one device copy
    if (m->vx.tp || m->vx.tp2) {
        VocRedoW rw;
        rw.M = cfg->mel_channels;
        rw.C = cfg->vocoder_channels;
        rw.wi = m->vin_w;
        rw.bi = m->vin_b;
        for (int k = 0; k < 4; ++k) {
            rw.wt[k] = m->up_w[k];
            rw.bt[k] = m->up_b[k];
            rw.w1[k] = m->rb_w1[k];
            rw.b1[k] = m->rb_b1[k];
            rw.w2[k] = m->rb_w2[k];
            rw.b2[k] = m->rb_b2[k];
        }
        rw.wo = m->vout_w;
        rw.bo = m->vout_b;
        void* dv = nullptr;
        e = hipMalloc(&dv, sizeof(VocRedoW));
        if (e == hipSuccess) e = hipMemcpyAsync(dv, &rw, sizeof(VocRedoW), hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            if (dv) (void)hipFree(dv);
            m2_model_destroy(m);
            return hip_status(e, "hipMalloc(redo weights)");
        }
        m->redo_w = static_cast<const VocRedoW*>(dv);
    }
    // work-queue counters of the one-launch transformer layers (TflQueue)
    // (+ 16 words: the count kernel's ticket of the device-T front half)
    e = hipMalloc(&m->tflq, (kTflQueueWords + 16) * sizeof(unsigned));
    if (e == hipSuccess) e = hipMemsetAsync(m->tflq, 0, (kTflQueueWords + 16) * sizeof(unsigned), st);
    if (e == hipSuccess) m->cnt_ticket = m->tflq + kTflQueueWords;
    if (e == hipSuccess) {
        void* h = nullptr;
        e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
        if (e == hipSuccess) {
            std::memset(h, 0, 64);
            m->fpost_host = static_cast<int32_t*>(h);
            void* d = nullptr;
            e = hipHostGetDevicePointer(&d, h, 0);
            m->fpost_dev = static_cast<int32_t*>(d);
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        m2_model_destroy(m);
        return hip_status(e, "hipMalloc(tfl queue)");
    }
    *out = m;
    return M2_OK;
}

int32_t m2_profile_disable(m2_model* model);

int32_t m2_model_destroy(m2_model* model) {
    if (!model) return M2_OK;
    m2_profile_disable(model);
    if (model->vbuf) (void)hipFree(model->vbuf);
    if (model->xbuf) (void)hipFree(model->xbuf);
    if (model->tbuf) (void)hipFree(model->tbuf);
    if (model->mbuf) (void)hipFree(model->mbuf);
    if (model->rflag_host) (void)hipHostFree(model->rflag_host);
    if (model->rflag_dev) (void)hipFree(model->rflag_dev);
    if (model->tflq) (void)hipFree(model->tflq);
    if (model->fpost_host) (void)hipHostFree(model->fpost_host);
    if (model->redo_w) (void)hipFree(const_cast<VocRedoW*>(model->redo_w));
    hipError_t e = hipFree(model->buf);
    delete model;
    if (e != hipSuccess) return hip_status(e, "hipFree(model)");
    return M2_OK;
}

int32_t m2_model_config(const m2_model* model, m2_config* out) {
    M2_CHECK_ARG(model && out, "m2_model_config: null argument");
    *out = model->cfg;
    return M2_OK;
}

size_t m2_workspace_bytes(const m2_model* model, int32_t B, int32_t S, int32_t T) {
    if (!model || B < 0 || S < 0 || T < 0) return 0;
    const int H = model->cfg.hidden_dim;
    Sizer a, b;
    carve_tf(a, B, S, H, model->cfg.num_heads, nullptr);
    carve_tf(b, B, T, H, model->cfg.num_heads, nullptr);
    return std::max(a.off, std::max(b.off, vocoder_ws_bytes(model, B, T))) + 256;
}

}  // extern "C"

namespace {
// TextEncoder.forward up to (not including) the final LayerNorm; *x_pre = the
// last layer's output in the workspace.
int32_t text_encoder_layers(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B, int32_t S,
                            uint8_t* out_mask, void* workspace, size_t workspace_bytes, hipStream_t st,
                            float** x_pre) {
    const int H = m->cfg.hidden_dim;
    Carve a(workspace, workspace_bytes);
    TfBufs wb;
    carve_tf(a, B, S, H, m->cfg.num_heads, &wb);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_text_encoder: workspace too small");
    *x_pre = wb.x;
    if (B == 0 || S == 0) return M2_OK;
    int32_t rc;
    const uint8_t* mask = nullptr;
    if (lengths) mask = out_mask ? out_mask : wb.mask;  // written by the embedding launch
    if (tfl_use(m, m->enc)) {
        const m2_layer_w& L0 = m->enc[0];
        TflFirst f;
        f.src = 1;
        f.ids = ids;
        f.emb = m->emb;
        f.pe = m->pe;
        f.vocab = m->cfg.vocab_size;
        f.escale = (float)std::sqrt((double)H);  // as launch_embed_pe
        f.lengths = lengths;
        f.mask = out_mask;
        if ((rc = launch_tfl_first(f, B, S, H, m->cfg.num_heads, lengths != nullptr, wb.x, L0.n1_w, L0.n1_b, L0.qkv_p,
                                   wb.tfl[0], tfl_queue(m), st)))
            return tfl_reset(m, st, rc);
        return run_tfl(m, m->enc, wb.x, wb.x, wb, lengths, B, S, st);
    }
    if (tf_first_fused(m, m->enc)) {
        const m2_layer_w& L0 = m->enc[0];
        if ((rc = launch_embed_ln_gemm(ids, m->emb, m->pe, B, S, H, m->cfg.vocab_size, lengths,
                                       const_cast<uint8_t*>(mask), wb.x, L0.n1_w, L0.n1_b, L0.qkv_p, 3 * H, wb.qkv,
                                       st)))
            return rc;
        return run_stack(m, m->enc, wb.x, wb.x, wb, mask, B, S, st, nullptr, nullptr, nullptr, nullptr, 0, nullptr,
                         nullptr, true);
    }
    if ((rc = launch_embed_pe(ids, m->emb, m->pe, B, S, H, m->cfg.vocab_size, wb.x, lengths,
                              const_cast<uint8_t*>(mask), st)))
        return rc;
    return run_stack(m, m->enc, wb.x, wb.x, wb, mask, B, S, st);
}
}  // namespace

extern "C" {

int32_t m2_text_encoder(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B,
                        int32_t S, float* out_enc, uint8_t* out_mask, void* workspace,
                        size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(m && ids && out_enc && B >= 0 && S >= 0, "m2_text_encoder: bad argument");
    M2_CHECK_SHAPE(S <= m->cfg.max_positions, "m2_text_encoder: sequence longer than the positional table");
    hipStream_t st = static_cast<hipStream_t>(stream);
    float* x = nullptr;
    int32_t rc = text_encoder_layers(m, ids, lengths, B, S, out_mask, workspace, workspace_bytes, st, &x);
    if (rc || B == 0 || S == 0) return rc;
    return launch_layer_norm(x, m->enc_nw, m->enc_nb, B * S, m->cfg.hidden_dim, out_enc, st);
}

int32_t m2_duration_predictor(const m2_model* m, const float* enc, int32_t B, int32_t S,
                              float* out_dur, void* workspace, size_t workspace_bytes, void* stream) {
    (void)workspace;
    (void)workspace_bytes;
    M2_CHECK_ARG(m && enc && out_dur && B >= 0 && S >= 0, "m2_duration_predictor: bad argument");
    return launch_duration(enc, B, S, m->cfg.hidden_dim, m->dur, out_dur, static_cast<hipStream_t>(stream));
}

int32_t m2_length_regulator_count(const void* dur, int32_t dur_is_int, float scale, int32_t B,
                                  int32_t S, int32_t* out_cum, int32_t* out_T, int32_t* out_Tmax,
                                  void* stream) {
    M2_CHECK_ARG(dur && out_cum && out_T && out_Tmax && B >= 0 && S >= 0, "m2_length_regulator_count: bad argument");
    return launch_lr_count(dur, dur_is_int, scale, B, S, out_cum, out_T, out_Tmax, static_cast<hipStream_t>(stream));
}

// Per-device mailbox of m2_length_regulator_count_sync: [seq, Tmax] in
// coherent host-mapped memory plus the count kernel's ticket counter.
namespace {
struct LrMailbox {
    int32_t* host = nullptr;
    int32_t* dev = nullptr;
    unsigned* ticket = nullptr;
    int32_t seq = 0;
};
constexpr int kMaxDevices = 64;
std::mutex g_mb_mu;
LrMailbox g_mb[kMaxDevices];

// The mailbox's device ticket is zeroed on the caller's stream `st` (and
// waited for): a blocking hipMemset would go to the null stream, which a
// non-blocking stream (e.g. a torch side stream) does not wait for, so the
// first count kernel could take its ticket before the zero landed and never
// post (seen as "stream idle but T_max not posted" on a first call from a
// side stream).
int32_t mailbox_for(int dev, hipStream_t st, LrMailbox** out) {
    LrMailbox& mb = g_mb[dev];
    if (!mb.host) {
        int cur = 0;
        M2_HIP(hipGetDevice(&cur));
        M2_HIP(hipSetDevice(dev));
        void* h = nullptr;
        hipError_t e = hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
        void* d = nullptr;
        if (e == hipSuccess) e = hipHostGetDevicePointer(&d, h, 0);
        void* t = nullptr;
        if (e == hipSuccess) e = hipMalloc(&t, sizeof(unsigned));
        (void)hipSetDevice(cur);
        if (e == hipSuccess) e = hipMemsetAsync(t, 0, sizeof(unsigned), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_status(e, "m2_length_regulator_count_sync: mailbox allocation");
        std::memset(h, 0, 64);
        mb.host = static_cast<int32_t*>(h);
        mb.dev = static_cast<int32_t*>(d);
        mb.ticket = static_cast<unsigned*>(t);
    }
    *out = &mb;
    return M2_OK;
}

// Spin on the mailbox until `seq` is posted; every 1024 polls ask the stream
// whether it failed (or finished without posting, which would be a bug).
int32_t mailbox_wait(const LrMailbox* mb, int32_t seq, hipStream_t st, int32_t* host_Tmax, const char* what) {
    for (unsigned i = 1;; ++i) {
        if (__atomic_load_n(mb->host, __ATOMIC_ACQUIRE) == seq) break;
        if ((i & 1023) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {
                if (__atomic_load_n(mb->host, __ATOMIC_ACQUIRE) == seq) break;
                return fail(M2_E_INTERNAL, (std::string(what) + ": stream idle but T_max not posted").c_str());
            }
            if (e != hipErrorNotReady) return hip_status(e, what);
        }
        _mm_pause();
    }
    *host_Tmax = __atomic_load_n(mb->host + 1, __ATOMIC_RELAXED);
    return M2_OK;
}

int32_t stream_device(hipStream_t st, int* dev) {
    if (st) M2_HIP(hipStreamGetDevice(st, dev));
    else M2_HIP(hipGetDevice(dev));
    M2_CHECK_ARG(*dev >= 0 && *dev < kMaxDevices, "T_max mailbox: device index");
    return M2_OK;
}
}  // namespace

int32_t m2_length_regulator_count_sync(const void* dur, int32_t dur_is_int, float scale, int32_t B, int32_t S,
                                       int32_t* out_cum, int32_t* out_T, int32_t* out_Tmax, int32_t* host_Tmax,
                                       void* stream) {
    M2_CHECK_ARG(out_Tmax && host_Tmax && B >= 0 && S >= 0, "m2_length_regulator_count_sync: bad argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (B == 0) {  // empty batch: the [0, ...] tensors have no storage
        M2_HIP(hipMemsetAsync(out_Tmax, 0, sizeof(int32_t), st));
        *host_Tmax = 0;
        return M2_OK;
    }
    M2_CHECK_ARG(dur && out_cum && out_T, "m2_length_regulator_count_sync: bad argument");
    int dev = 0;
    int32_t rc0 = stream_device(st, &dev);
    if (rc0) return rc0;
    std::lock_guard<std::mutex> lk(g_mb_mu);
    LrMailbox* mb = nullptr;
    int32_t rc = mailbox_for(dev, st, &mb);
    if (rc) return rc;
    mb->seq = mb->seq == INT_MAX ? 1 : mb->seq + 1;
    const int32_t seq = mb->seq;
    if ((rc = launch_lr_count_sync(dur, dur_is_int, scale, B, S, out_cum, out_T, out_Tmax, mb->ticket, mb->dev, seq,
                                   st)))
        return rc;
    if ((rc = mailbox_wait(mb, seq, st, host_Tmax, "m2_length_regulator_count_sync"))) return rc;
    M2_CHECK_SHAPE(*host_Tmax <= kMaxFrames, "length regulator: an utterance's frame count exceeds 2^24 (the "
                                             "durations times duration_scale are out of range)");
    return M2_OK;
}

int32_t m2_length_regulator_expand(const float* enc, const int32_t* cum, int32_t B, int32_t S,
                                   int32_t H, int32_t T_out, float* out, void* stream) {
    M2_CHECK_ARG(enc && cum && out && B >= 0 && S >= 0 && H > 0 && T_out >= 0, "m2_length_regulator_expand: bad argument");
    return launch_lr_expand(enc, cum, B, S, H, T_out, out, static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {
// The mel decoder on x [B, T, H]; with enc / cum given, x is first filled by
// the length regulator's frame expansion of enc, fused into the first layer's
// LN1 -> QKV launch when tf_first_fused (else a separate lr_expand launch).
int32_t mel_decoder(const m2_model* m, float* x, int32_t B, int32_t T, float* out_mel, void* workspace,
                    size_t workspace_bytes, hipStream_t st, const float* enc = nullptr, const int32_t* cum = nullptr,
                    int32_t S = 0, const int32_t* dT = nullptr) {
    const int H = m->cfg.hidden_dim;
    Carve a(workspace, workspace_bytes);
    TfBufs wb;
    carve_tf(a, B, T, H, m->cfg.num_heads, &wb);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_mel_decoder: workspace too small");
    if (B == 0 || T == 0) return M2_OK;
    int32_t rc;
    // dT: T is the capacity of a speculative launch (spec_ok: one-launch
    // layers with the mel projection fused into the last one)
    M2_CHECK_ARG(!dT || (tfl_use(m, m->dec) && tfl_proj_supported(H, m->cfg.mel_channels)),
                 "mel decoder: a device frame count needs the one-launch layers");
    if (tfl_use(m, m->dec)) {
        const m2_layer_w& L0 = m->dec[0];
        TflFirst f;
        f.dN = dT;
        if (dT) {  // the first launch posts T for the host (m2_frames_wait)
            m->fpost_seq = m->fpost_seq == INT_MAX ? 1 : m->fpost_seq + 1;
            f.post = m->fpost_dev;
            f.post_seq = m->fpost_seq;
        }
        if (enc) {  // the length regulator's expansion, built by the first launch into x
            f.src = 2;
            f.enc = enc;
            f.cum = cum;
            f.S = S;
        } else {
            f.src = 0;
            f.x_in = x;
        }
        if ((rc = launch_tfl_first(f, B, T, H, m->cfg.num_heads, false, x, L0.n1_w, L0.n1_b, L0.qkv_p, wb.tfl[0],
                                   tfl_queue(m), st)))
            return tfl_reset(m, st, rc);
        bool projected = false;
        if ((rc = run_tfl(m, m->dec, x, wb.x, wb, nullptr, B, T, st, m->dec_nw, m->dec_nb, m->mel_p, m->mel_b,
                          m->cfg.mel_channels, out_mel, &projected, dT)))
            return rc;
        if (projected) return M2_OK;
        return launch_ln_gemm(wb.x, m->dec_nw, m->dec_nb, m->mel_p, m->mel_b, ACT_NONE, B * T, H, m->cfg.mel_channels,
                              out_mel, st);
    }
    bool qkv_ready = false;
    if (enc) {
        if (tf_first_fused(m, m->dec)) {
            const m2_layer_w& L0 = m->dec[0];
            if ((rc = launch_expand_ln_gemm(enc, cum, B, S, T, H, x, L0.n1_w, L0.n1_b, L0.qkv_p, 3 * H, wb.qkv, st)))
                return rc;
            qkv_ready = true;
        } else if ((rc = launch_lr_expand(enc, cum, B, S, H, T, x, st))) {
            return rc;
        }
    }
    bool projected = false;
    if ((rc = run_stack(m, m->dec, x, wb.x, wb, nullptr, B, T, st, m->dec_nw, m->dec_nb, m->mel_p, m->mel_b,
                        m->cfg.mel_channels, out_mel, &projected, qkv_ready)))
        return rc;
    if (projected) return M2_OK;
    const float* cur = m->dec.empty() ? x : wb.x;
    if (m->tfused)
        return launch_ln_gemm(cur, m->dec_nw, m->dec_nb, m->mel_p, m->mel_b, ACT_NONE, B * T, H, m->cfg.mel_channels,
                              out_mel, st);
    return launch_linear(cur, m->dec_nw, m->dec_nb, m->mel_w, m->mel_b, nullptr, ACT_NONE, B * T, H,
                         m->cfg.mel_channels, out_mel, st);
}
}  // namespace

extern "C" {

int32_t m2_mel_decoder(const m2_model* m, const float* x, int32_t B, int32_t T, float* out_mel,
                       void* workspace, size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(m && x && out_mel && B >= 0 && T >= 0, "m2_mel_decoder: bad argument");
    return mel_decoder(m, const_cast<float*>(x), B, T, out_mel, workspace, workspace_bytes,
                       static_cast<hipStream_t>(stream));
}

}  // extern "C"

namespace {
int32_t vocoder_run(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T, float* out_audio,
                    float* const* buf, hipStream_t st, bool x3, int redo = -1, const int32_t* dT = nullptr);

// Audio samples [64 f0, 64 f1) of every utterance of a T-frame mel, computed
// over the window [f0 - halo, f1 + halo) clipped to [0, T): the window's mel
// rows are copied to c.mel (same layout, T_w frames), vocoded as a T_w-frame
// call, and the centre of its audio copied to out (row pitch out_pitch floats,
// utterance b's chunk at out + b * out_pitch).
int32_t vocoder_window(const m2_model* m, const float* mel, int32_t layout, int32_t B, int32_t T, int32_t f0,
                       int32_t f1, float* out, size_t out_pitch, const ChunkBufs& c, hipStream_t st, bool x3,
                       int redo = -1) {
    const int M = m->cfg.mel_channels;
    const int w0 = std::max(0, f0 - kVocHalo), w1 = std::min(T, f1 + kVocHalo), W = w1 - w0;
    if (layout == 1)  // [B,T,M]: utterance b's window is W*M contiguous floats
        M2_HIP(hipMemcpy2DAsync(c.mel, (size_t)W * M * 4, mel + (size_t)w0 * M, (size_t)T * M * 4, (size_t)W * M * 4, B,
                                hipMemcpyDeviceToDevice, st));
    else  // [B,M,T]: one W-float row per (utterance, channel)
        M2_HIP(hipMemcpy2DAsync(c.mel, (size_t)W * 4, mel + w0, (size_t)T * 4, (size_t)W * 4, (size_t)B * M,
                                hipMemcpyDeviceToDevice, st));
    int32_t rc = vocoder_run(m, c.mel, layout, B, W, c.audio, c.voc, st, x3, redo);
    if (rc) return rc;
    M2_HIP(hipMemcpy2DAsync(out, out_pitch * 4, c.audio + (size_t)64 * (f0 - w0), (size_t)64 * W * 4,
                            (size_t)64 * (f1 - f0) * 4, B, hipMemcpyDeviceToDevice, st));
    return M2_OK;
}

// One m2_vocoder call on the split (x3) or exact-f32 kernels; redo >= 0: the
// on-device range redo with flag word redo (vocoder_run).
int32_t vocoder_call(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T, float* out_audio,
                     void* workspace, size_t workspace_bytes, hipStream_t st, bool x3, int redo = -1,
                     const int32_t* dT = nullptr) {
    Carve a(workspace, workspace_bytes);
    M2_CHECK_ARG(!dT || (m->fused && !(m->chunk_frames > 0 && T > m->chunk_frames)),
                 "m2_vocoder: a device frame count needs the fused, unchunked vocoder");
    if (m->chunk_frames > 0 && T > m->chunk_frames) {  // streamed: chunk by chunk into out_audio
        ChunkBufs c;
        carve_chunked(a, m->cfg, B, T, m->chunk_frames, &c);
        if (!a.ok) return fail(M2_E_WORKSPACE, "m2_vocoder: workspace too small");
        if (B == 0) return M2_OK;
        for (int f0 = 0; f0 < T; f0 += m->chunk_frames) {
            const int f1 = std::min(T, f0 + m->chunk_frames);
            const int32_t rc = vocoder_window(m, mel, mel_layout, B, T, f0, f1, out_audio + (size_t)64 * f0,
                                              (size_t)64 * T, c, st, x3, redo);
            if (rc) return rc;
        }
        return M2_OK;
    }
    float* buf[3];
    carve_voc(a, m->cfg, B, T, buf);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_vocoder: workspace too small");
    if (B == 0 || T == 0) return M2_OK;
    return vocoder_run(m, mel, mel_layout, B, T, out_audio, buf, st, x3, redo, dT);
}

// Sticky range error of an earlier call (policy 0), returned and cleared on entry.
int32_t range_entry(const m2_model* m, const char* what) {
    if (m->rflag_host && __atomic_load_n(m->rflag_host, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(m->rflag_host, 0, __ATOMIC_RELEASE);
        return fail(M2_E_RANGE, (std::string(what) + ": an earlier vocoder call on this model produced non-finite "
                                 "audio on the split-f16 path (an input or activation of magnitude >= 65520, or "
                                 "a non-finite input); its output is invalid - re-run it with "
                                 "m2_vocoder_select(model, 1) or range policy 1").c_str());
    }
    return M2_OK;
}

// Policy 1 on the fused vocoders: the flag word of this call for an on-device
// redo (vocoder_run), or -1 (the host-side fallback below).
int device_redo_word(const m2_model* m, bool x3) {
    if (m->range_policy != 1 || !x3 || !m->fused || !m->rflag_dev) return -1;
    return (int)(m->rseq++ & 1u);
}

// Policy 1 otherwise: wait for the call, and re-run it on the exact-f32
// kernels if its audio came out non-finite.
template <typename F>
int32_t range_fallback(const m2_model* m, hipStream_t st, bool x3, F redo) {
    if (m->range_policy != 1 || !x3 || !m->rflag_host) return M2_OK;
    M2_HIP(hipStreamSynchronize(st));
    if (!__atomic_load_n(m->rflag_host, __ATOMIC_ACQUIRE)) return M2_OK;
    __atomic_store_n(m->rflag_host, 0, __ATOMIC_RELEASE);
    return redo();
}

// m2_vocoder; dT: T is the capacity of a speculative launch (dev_frames)
int32_t vocoder_entry(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T, float* out_audio,
                      void* workspace, size_t workspace_bytes, void* stream, const int32_t* dT = nullptr) {
    M2_CHECK_ARG(m && mel && out_audio && B >= 0 && T >= 0, "m2_vocoder: bad argument");
    M2_CHECK_ARG(mel_layout == 0 || mel_layout == 1, "m2_vocoder: mel_layout must be 0 or 1");
    hipStream_t st = static_cast<hipStream_t>(stream);
    int32_t rc = range_entry(m, "m2_vocoder");
    if (rc) return rc;
    const bool x3 = m->x3;
    const int redo = device_redo_word(m, x3);
    if ((rc = vocoder_call(m, mel, mel_layout, B, T, out_audio, workspace, workspace_bytes, st, x3, redo, dT)))
        return rc;
    if (redo >= 0) return M2_OK;
    return range_fallback(m, st, x3, [&] {
        return vocoder_call(m, mel, mel_layout, B, T, out_audio, workspace, workspace_bytes, st, false, -1, dT);
    });
}
}  // namespace

extern "C" {

int32_t m2_vocoder(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T,
                   float* out_audio, void* workspace, size_t workspace_bytes, void* stream) {
    return vocoder_entry(m, mel, mel_layout, B, T, out_audio, workspace, workspace_bytes, stream);
}

int32_t m2_vocoder_chunk(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T, int32_t f0,
                         int32_t f1, float* out_chunk, void* workspace, size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(m && mel && out_chunk && B >= 0 && T >= 0, "m2_vocoder_chunk: bad argument");
    M2_CHECK_ARG(mel_layout == 0 || mel_layout == 1, "m2_vocoder_chunk: mel_layout must be 0 or 1");
    M2_CHECK_ARG(0 <= f0 && f0 < f1 && f1 <= T, "m2_vocoder_chunk: need 0 <= f0 < f1 <= T");
    int32_t rc = range_entry(m, "m2_vocoder_chunk");
    if (rc) return rc;
    Carve a(workspace, workspace_bytes);
    ChunkBufs c;
    carve_chunked(a, m->cfg, B, T, f1 - f0, &c);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_vocoder_chunk: workspace too small");
    if (B == 0) return M2_OK;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const bool x3 = m->x3;
    const int redo = device_redo_word(m, x3);
    if ((rc = vocoder_window(m, mel, mel_layout, B, T, f0, f1, out_chunk, (size_t)64 * (f1 - f0), c, st, x3, redo)))
        return rc;
    if (redo >= 0) return M2_OK;
    return range_fallback(m, st, x3, [&] {
        return vocoder_window(m, mel, mel_layout, B, T, f0, f1, out_chunk, (size_t)64 * (f1 - f0), c, st, false);
    });
}

int32_t m2_set_range_policy(m2_model* m, int32_t policy) {
    M2_CHECK_ARG(m && (policy == 0 || policy == 1), "m2_set_range_policy: policy must be 0 (report) or 1 (fallback)");
    m->range_policy = policy;
    return M2_OK;
}

int32_t m2_model_check(m2_model* m, void* stream, int32_t* flagged) {
    M2_CHECK_ARG(m && flagged, "m2_model_check: bad argument");
    M2_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    *flagged = m->rflag_host ? __atomic_exchange_n(m->rflag_host, 0, __ATOMIC_ACQ_REL) : 0;
    return M2_OK;
}

size_t m2_vocoder_chunk_workspace_bytes(const m2_model* m, int32_t B, int32_t T, int32_t chunk_frames) {
    if (!m || B < 0 || T < 0 || chunk_frames <= 0) return 0;
    Sizer s;
    carve_chunked(s, m->cfg, B, T, chunk_frames, nullptr);
    return s.off + 256;
}

int32_t m2_vocoder_set_chunking(m2_model* m, int32_t chunk_frames) {
    M2_CHECK_ARG(m && chunk_frames >= 0, "m2_vocoder_set_chunking: bad argument");
    m->chunk_frames = chunk_frames;
    return M2_OK;
}

int32_t m2_vocoder_halo_frames(void) { return kVocHalo; }

int32_t m2_vocoder_select(m2_model* m, int32_t path) {
    M2_CHECK_ARG(m, "m2_vocoder_select: null model");
    if (path == 2) {
        M2_CHECK_ARG(m->x3_packed, "m2_vocoder_select: no split-f16 packs (shape unsupported, weights outside the "
                                   "f16 range or M2_VOC_F32 set at creation)");
        m->x3 = true;
        return M2_OK;
    }
    M2_CHECK_ARG(path == 1 && m->fused, "m2_vocoder_select: path must be 1 (exact-f32) or 2 (split-f16)");
    m->x3 = false;
    return M2_OK;
}

}  // extern "C"

namespace {
// redo >= 0 (range policy 1, x3): the split kernels raise flag word `redo`
// instead of the host-mapped flag, and the exact-f32 kernels follow, each
// workgroup returning at once unless that word is raised - a call whose split
// audio came out non-finite is recomputed on the device, with no host wait.
int32_t vocoder_run(const m2_model* m, const float* mel, int32_t mel_layout, int32_t B, int32_t T, float* out_audio,
                    float* const* buf, hipStream_t st, bool x3, int redo, const int32_t* dT) {
    int32_t rc;
    if (m->fused) {
        const int call = m->prof_calls;
        const bool rec = (size_t)(call + 1) * kVocKernels <= m->prof_begin.size() &&
                         m->prof_seen++ % m->prof_stride == 0;
        if (rec) m->prof_calls++;
        auto mark = [&](int kidx, bool begin) {
            if (!rec || !((m->prof_mask >> kidx) & 1u)) return;
            const size_t slot = (size_t)call * kVocKernels + kidx;
            (void)hipEventRecord(begin ? m->prof_begin[slot] : m->prof_end[slot], st);
        };
        VocX vx = m->vx;
        VocW vw = m->vw;
        vx.dT = vw.dT = dT;
        vx.head_prio = sw().x3_head_prio;
        if (x3 && redo >= 0) {
            vx.rflag = m->rflag_dev + redo;
            vx.rclear = m->rflag_dev + (redo ^ 1);
            vx.rqueue = reinterpret_cast<unsigned*>(m->rflag_dev + 4);
            if (m->redo_w && !sw().redo_launch) {
                // the pipelined tail redoes its own non-finite strips
                // in fp32 inside the launch: no guarded launch behind it
                vx.redo_w = m->redo_w;
                return launch_vocoder_x3(mel, mel_layout == 1, m->cfg.mel_channels, m->cfg.vocoder_channels, B, T,
                                         vx, buf[0], buf[1], out_audio, st, mark);
            }
            if ((rc = launch_vocoder_x3(mel, mel_layout == 1, m->cfg.mel_channels, m->cfg.vocoder_channels, B, T, vx,
                                        buf[0], buf[1], out_audio, st, mark)))
                return rc;
            vw.guard = m->rflag_dev + redo;
            vw.guard_queue = reinterpret_cast<const unsigned*>(m->rflag_dev + 4);  // words 4-7 (zeroed by the head)
            return launch_vocoder_fused(mel, mel_layout == 1, m->cfg.mel_channels, m->cfg.vocoder_channels, B, T, vw,
                                        buf[0], buf[1], out_audio, st, [](int, bool) {});
        }
        if (x3)
            return launch_vocoder_x3(mel, mel_layout == 1, m->cfg.mel_channels, m->cfg.vocoder_channels, B, T, vx,
                                     buf[0], buf[1], out_audio, st, mark);
        return launch_vocoder_fused(mel, mel_layout == 1, m->cfg.mel_channels, m->cfg.vocoder_channels, B, T, vw,
                                    buf[0], buf[1], out_audio, st, mark);
    }
    M2_CHECK_ARG(!dT, "m2_vocoder: a device frame count needs the fused vocoder");
    int ch = m->cfg.vocoder_channels, L = T;
    float *cur = buf[0], *up = buf[1], *tmp = buf[2];
    if ((rc = launch_conv(mel, m->vin_w, m->vin_b, nullptr, nullptr, nullptr, 3, ACT_NONE, mel_layout == 1, B, m->cfg.mel_channels, ch, L, cur, st))) return rc;
    for (int k = 0; k < 4; ++k) {
        if ((rc = launch_convT(cur, m->up_w[k], m->up_b[k], kRates[k], ACT_LEAKY, B, ch, ch / 2, L, up, st))) return rc;
        ch /= 2;
        L *= kRates[k];
        if ((rc = launch_conv(up, m->rb_w1[k], m->rb_b1[k], nullptr, nullptr, nullptr, 3, ACT_LEAKY, false, B, ch, ch, L, tmp, st))) return rc;
        if ((rc = launch_conv(tmp, m->rb_w2[k], m->rb_b2[k], nullptr, nullptr, up, 3, ACT_NONE, false, B, ch, ch, L, cur, st))) return rc;
    }
    return launch_conv(cur, m->vout_w, m->vout_b, nullptr, nullptr, nullptr, 3, ACT_TANH, false, B, ch, 1, L, out_audio, st);
}
}  // namespace

extern "C" {

int32_t m2_vocoder_resblock(const m2_model* m, int32_t k, const float* x, int32_t B, int32_t L,
                            float* y, float* tmp, void* stream) {
    M2_CHECK_ARG(m && x && y && tmp && k >= 0 && k < 4 && B >= 0 && L >= 0, "m2_vocoder_resblock: bad argument");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int ch = m->cfg.vocoder_channels >> (k + 1);
    int32_t rc;
    if ((rc = launch_conv(x, m->rb_w1[k], m->rb_b1[k], nullptr, nullptr, nullptr, 3, ACT_LEAKY, false, B, ch, ch, L, tmp, st))) return rc;
    return launch_conv(tmp, m->rb_w2[k], m->rb_b2[k], nullptr, nullptr, x, 3, ACT_NONE, false, B, ch, ch, L, y, st);
}

int32_t m2_vocoder_upsample(const m2_model* m, int32_t k, const float* x, int32_t B, int32_t L,
                            float* y, void* stream) {
    M2_CHECK_ARG(m && x && y && k >= 0 && k < 4 && B >= 0 && L >= 0, "m2_vocoder_upsample: bad argument");
    const int ch = m->cfg.vocoder_channels >> k;
    return launch_convT(x, m->up_w[k], m->up_b[k], kRates[k], ACT_LEAKY, B, ch, ch / 2, L, y, static_cast<hipStream_t>(stream));
}

int32_t m2_conv1d(const float* x, const float* w, const float* b, const float* alpha,
                  const float* beta, const float* res, int32_t ksize, int32_t act, int32_t B,
                  int32_t Cin, int32_t Cout, int32_t L, float* y, void* stream) {
    M2_CHECK_ARG(x && w && b && y && B >= 0 && L >= 0 && act >= 0 && act <= 4, "m2_conv1d: bad argument");
    return launch_conv(x, w, b, alpha, beta, res, ksize, act, false, B, Cin, Cout, L, y, static_cast<hipStream_t>(stream));
}

int32_t m2_conv1d_ex(const float* x, const float* w, const float* b, const float* alpha, const float* beta,
                     const float* res, int32_t ksize, int32_t dilation, int32_t padding, int32_t act, int32_t B,
                     int32_t Cin, int32_t Cout, int32_t L, float* y, void* stream) {
    M2_CHECK_ARG(x && w && b && y && B >= 0 && L >= 0, "m2_conv1d_ex: bad argument");
    return launch_conv_general(x, w, b, alpha, beta, res, ksize, dilation, padding, act, B, Cin, Cout, L, y,
                               static_cast<hipStream_t>(stream));
}

int32_t m2_conv_transpose1d(const float* x, const float* w, const float* b, int32_t rate,
                            int32_t act, int32_t B, int32_t Cin, int32_t Cout, int32_t L, float* y,
                            void* stream) {
    M2_CHECK_ARG(x && w && b && y && B >= 0 && L >= 0 && act >= 0 && act <= 3, "m2_conv_transpose1d: bad argument");
    return launch_convT(x, w, b, rate, act, B, Cin, Cout, L, y, static_cast<hipStream_t>(stream));
}

int32_t m2_linear(const float* x, const float* gamma, const float* beta, const float* w,
                  const float* b, const float* res, int32_t act, int32_t R, int32_t K, int32_t N,
                  float* y, void* stream) {
    M2_CHECK_ARG(x && w && y && R >= 0 && (act == ACT_NONE || act == ACT_RELU), "m2_linear: bad argument");
    M2_CHECK_ARG((gamma == nullptr) == (beta == nullptr), "m2_linear: gamma and beta go together");
    return launch_linear(x, gamma, beta, w, b, res, act, R, K, N, y, static_cast<hipStream_t>(stream));
}

int32_t m2_layer_norm(const float* x, const float* gamma, const float* beta, int32_t R, int32_t K,
                      float* y, void* stream) {
    M2_CHECK_ARG(x && gamma && beta && y && R >= 0 && K > 0, "m2_layer_norm: bad argument");
    return launch_layer_norm(x, gamma, beta, R, K, y, static_cast<hipStream_t>(stream));
}

int32_t m2_attention(const float* qkv, const uint8_t* key_mask, int32_t B, int32_t N, int32_t H,
                     int32_t heads, float* out, void* stream) {
    M2_CHECK_ARG(qkv && out && B >= 0 && N >= 0 && H > 0 && heads > 0, "m2_attention: bad argument");
    return launch_attention(qkv, key_mask, B, N, H, heads, out, static_cast<hipStream_t>(stream));
}

int32_t m2_embed_positional(const int64_t* ids, const float* emb, const float* pe, int32_t B,
                            int32_t S, int32_t H, int32_t vocab, float scale, float* y,
                            void* stream) {
    M2_CHECK_ARG(ids && emb && pe && y && B >= 0 && S >= 0 && H > 0 && vocab > 0, "m2_embed_positional: bad argument");
    return launch_embed_pe_scaled(ids, emb, pe, B, S, H, vocab, scale, y, static_cast<hipStream_t>(stream));
}

int32_t m2_add_positional(const float* x, const float* pe, int32_t B, int32_t S, int32_t H,
                          float* y, void* stream) {
    M2_CHECK_ARG(x && pe && y && B >= 0 && S >= 0 && H > 0, "m2_add_positional: bad argument");
    return launch_add_pe(x, pe, B, S, H, y, static_cast<hipStream_t>(stream));
}

int32_t m2_profile_kernel_count(void) { return kVocKernels; }

const char* m2_profile_kernel_name(int32_t index) {
    return (index >= 0 && index < kVocKernels) ? kVocKernelNames[index] : "";
}

const char* m2_profile_kernel_name_for(const m2_model* m, int32_t index) {
    if (!m || index < 0 || index >= kVocKernels) return "";
    if (m->x3 && m->tailp && index == 2) return m->vx.tp2 ? kVocTailp2KernelName : kVocTailpKernelName;
    if (m->x3 && m->midp && index == 1) return kVocMidpKernelName;
    return m->x3 ? kVocX3KernelNames[index] : kVocKernelNames[index];
}

size_t m2_front_bytes(const m2_model* model, int32_t B, int32_t S) {
    if (!model || B < 0 || S < 0) return 0;
    Sizer a;
    carve_front(a, B, S, model->cfg.hidden_dim, nullptr);
    return a.off + 256;
}

}  // extern "C"

namespace {
// The front half up to the frame counts: encoder, durations (into f), then
// the frame counts.  With `fuse` (and a batch small enough, fuse_count) the
// duration kernel's last workgroup runs the count itself: T_max into fuse->Tmax, the ticket
// fuse->ticket, the optional mailbox post; otherwise count(f) launches the
// length regulator's count kernel.
struct CountFuse {
    float scale;
    int32_t* Tmax;  // null: the front buffer's own T_max word
    unsigned* ticket;
    int32_t* mbox;
    int32_t seq;
};
// Default: fused for B * S <= 2048.  The last workgroup's count is serial
// work behind every other workgroup: at stage2 B=8 S=100 the step is 1.9 %
// shorter fused (duration 13.3 -> 15.7 us, the 5 us count launch gone), at
// stage1 B=32 and stage2 B=64 S=100 it measured +0.3 / +0.7 % (in-process
// A/B, profiles/r03/r03aa_ab.txt; again on the round-6 tree, stage1 B=32
// S=100: 0.1455 -> 0.1469 ms fused, profiles/r06/r06z12_count_ab.txt).
// M2_DUR_COUNT=1 fuses up to the kernel's limit (8192), =0 never.
bool fuse_count(int B, int S) {
    if (sw().dur_count >= 0) return sw().dur_count != 0 && duration_count_fusable(B, S);
    return (long)B * S <= 2048 && duration_count_fusable(B, S);
}
template <typename Count>
int32_t front_run(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B, int32_t S, void* front,
                  size_t front_bytes, void* workspace, size_t workspace_bytes, hipStream_t st, FrontBufs* f,
                  Count count, const CountFuse* fuse = nullptr) {
    M2_CHECK_ARG(m && B >= 0 && S >= 0, "m2_inference_front: bad argument");
    M2_CHECK_ARG(ids || B * S == 0, "m2_inference_front: null ids");
    if (int32_t rc0 = range_entry(m, "m2_inference")) return rc0;
    Carve a(front, front_bytes);
    carve_front(a, B, S, m->cfg.hidden_dim, f);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_inference_front: front buffer too small");
    int32_t rc;
    if (B > 0 && S > 0) {
        M2_CHECK_SHAPE(S <= m->cfg.max_positions, "m2_inference: sequence longer than the positional table");
        float* x = nullptr;
        if ((rc = text_encoder_layers(m, ids, lengths, B, S, lengths ? f->mask : nullptr, workspace, workspace_bytes,
                                      st, &x)))
            return rc;
        // the encoder's final LayerNorm runs inside the duration kernel, which
        // also stores the normalised encoder output (f.enc)
        // (split-f16 convs when the static range bound allows: dur_split)
        const float* const* ws = m->dur_split && sw().dur_split ? m->dur_split_w : nullptr;
        if (fuse && fuse_count(B, S))
            return launch_duration_count(x, B, S, m->cfg.hidden_dim, m->dur, f->dur, st, m->enc_nw, m->enc_nb, f->enc,
                                         fuse->scale, f->cum, f->tot, fuse->Tmax ? fuse->Tmax : f->tmax,
                                         fuse->ticket, fuse->mbox, fuse->seq, ws);
        if ((rc = launch_duration(x, B, S, m->cfg.hidden_dim, m->dur, f->dur, st, m->enc_nw, m->enc_nb, f->enc, ws)))
            return rc;
    }
    // Round 1's fused count (per-utterance tickets behind release fences: one
    // L2 write-back per workgroup) measured 5 us slower than this separate
    // kernel (tools/probe/count_fusion_ab.py, r17); the fused form above hands
    // the durations over with write-through stores instead.
    return count(*f);
}

// The back half can run from a device-resident frame count with its grids
// sized for T_cap frames: the one-launch decoder layers with the mel
// projection fused into the last one, and the fused (unchunked) vocoder.
bool dev_back_ok(const m2_model* m, int32_t T_cap) {
    if (!sw().speculative) return false;  // M2_SPECULATIVE=0: host-side T only (A/B, tests)
    return T_cap > 0 && tfl_use(m, m->dec) && tfl_proj_supported(m->cfg.hidden_dim, m->cfg.mel_channels) &&
           m->fused && !(m->chunk_frames > 0 && T_cap > m->chunk_frames);
}

// expansion to T frames + decoder + vocoder; dT: T is the capacity and the
// kernels take the frame count from the device word (dev_frames)
int32_t back_run(const m2_model* m, int32_t B, int32_t S, int32_t T, const int32_t* dT, const void* front,
                 size_t front_bytes, float* out_mel, float* out_audio, void* workspace, size_t workspace_bytes,
                 void* stream) {
    M2_CHECK_ARG(m && B >= 0 && S >= 0 && T >= 0, "m2_inference_back: bad argument");
    if (B == 0 || T == 0) return M2_OK;
    M2_CHECK_ARG(out_mel && out_audio, "m2_inference_back: null output");
    const int H = m->cfg.hidden_dim;
    Carve a(const_cast<void*>(front), front_bytes);
    FrontBufs f;
    carve_front(a, B, S, H, &f);
    if (!a.ok) return fail(M2_E_WORKSPACE, "m2_inference_back: front buffer too small");
    // the regulated frames live after the decoder / vocoder scratch
    Carve w(workspace, workspace_bytes);
    Sizer sz_tf;
    carve_tf(sz_tf, B, T, H, m->cfg.num_heads, nullptr);
    const size_t scratch = std::max(sz_tf.off, vocoder_ws_bytes(m, B, T));
    (void)w.take<char>(scratch);
    float* reg = w.take<float>((size_t)B * T * H);
    if (!w.ok) return fail(M2_E_WORKSPACE, "m2_inference_back: workspace too small");
    int32_t rc;
    // frame expansion + decoder (the expansion fused into the first layer's launch)
    if ((rc = mel_decoder(m, reg, B, T, out_mel, workspace, scratch, static_cast<hipStream_t>(stream), f.enc, f.cum,
                          S, dT)))
        return rc;
    return vocoder_entry(m, out_mel, 1, B, T, out_audio, workspace, scratch, stream, dT);
}
}  // namespace

extern "C" {

int32_t m2_inference_front(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B, int32_t S,
                           float scale, void* front, size_t front_bytes, void* workspace, size_t workspace_bytes,
                           int32_t* host_Tmax, void* stream) {
    M2_CHECK_ARG(host_Tmax, "m2_inference_front: bad argument");
    FrontBufs f;
    return front_run(m, ids, lengths, B, S, front, front_bytes, workspace, workspace_bytes,
                     static_cast<hipStream_t>(stream), &f, [&](FrontBufs& fb) {
                         return m2_length_regulator_count_sync(fb.dur, 0, scale, B, S, fb.cum, fb.tot, fb.tmax,
                                                               host_Tmax, stream);
                     });
}

int32_t m2_inference_front_dev(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B, int32_t S,
                               float scale, void* front, size_t front_bytes, void* workspace, size_t workspace_bytes,
                               int32_t* dev_Tmax, void* stream) {
    M2_CHECK_ARG(dev_Tmax, "m2_inference_front_dev: null T_max word");
    hipStream_t st = static_cast<hipStream_t>(stream);
    FrontBufs f;
    const CountFuse cf{scale, dev_Tmax, m->cnt_ticket, nullptr, 0};
    return front_run(m, ids, lengths, B, S, front, front_bytes, workspace, workspace_bytes, st, &f,
                     [&](FrontBufs& fb) -> int32_t {
                         if (B == 0) {
                             M2_HIP(hipMemsetAsync(dev_Tmax, 0, sizeof(int32_t), st));
                             return M2_OK;
                         }
                         return launch_lr_count_sync(fb.dur, 0, scale, B, S, fb.cum, fb.tot, dev_Tmax,
                                                     m->cnt_ticket, nullptr, 0, st);
                     }, &cf);
}

int32_t m2_inference_back(const m2_model* m, int32_t B, int32_t S, int32_t T, const void* front, size_t front_bytes,
                          float* out_mel, float* out_audio, void* workspace, size_t workspace_bytes, void* stream) {
    return back_run(m, B, S, T, nullptr, front, front_bytes, out_mel, out_audio, workspace, workspace_bytes, stream);
}

int32_t m2_inference_dev_supported(const m2_model* m, int32_t T_cap) { return m && dev_back_ok(m, T_cap) ? 1 : 0; }

int32_t m2_inference_back_dev(const m2_model* m, int32_t B, int32_t S, int32_t T_cap, const int32_t* dev_T,
                              const void* front, size_t front_bytes, float* out_mel, float* out_audio,
                              void* workspace, size_t workspace_bytes, void* stream) {
    M2_CHECK_ARG(m && dev_T && T_cap > 0, "m2_inference_back_dev: bad argument");
    M2_CHECK_ARG(dev_back_ok(m, T_cap), "m2_inference_back_dev: this model's back half needs the host-side frame "
                                        "count (m2_inference_dev_supported is 0)");
    return back_run(m, B, S, T_cap, dev_T, front, front_bytes, out_mel, out_audio, workspace, workspace_bytes, stream);
}

int32_t m2_frames_wait(const m2_model* m, void* stream, int32_t* host_T) {
    M2_CHECK_ARG(m && host_T, "m2_frames_wait: bad argument");
    M2_CHECK_ARG(m->fpost_seq > 0, "m2_frames_wait: no m2_inference_back_dev call to wait for");
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int32_t seq = m->fpost_seq;
    for (unsigned i = 1;; ++i) {
        if (__atomic_load_n(m->fpost_host, __ATOMIC_ACQUIRE) == seq) break;
        if ((i & 1023) == 0) {
            const hipError_t e = hipStreamQuery(st);
            if (e == hipSuccess) {
                if (__atomic_load_n(m->fpost_host, __ATOMIC_ACQUIRE) == seq) break;
                return fail(M2_E_INTERNAL, "m2_frames_wait: stream idle but T not posted");
            }
            if (e != hipErrorNotReady) return hip_status(e, "m2_frames_wait");
        }
        _mm_pause();
    }
    *host_T = __atomic_load_n(m->fpost_host + 1, __ATOMIC_RELAXED);
    return M2_OK;
}

int32_t m2_inference(const m2_model* m, const int64_t* ids, const int64_t* lengths, int32_t B, int32_t S, float scale,
                     void* front, size_t front_bytes, void* workspace, size_t workspace_bytes, float* mel_buf,
                     size_t mel_cap, float* audio_buf, size_t audio_cap, int32_t* host_T, int32_t* launched,
                     void* stream) {
    M2_CHECK_ARG(m && host_T && launched, "m2_inference: bad argument");
    *launched = 0;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // The capacity the caller's buffers give: with one, the back half is
    // enqueued right behind the count kernel, before the host reads T_max,
    // its kernels taking the frame count from the device (dev_frames) - the
    // host wait overlaps the decoder instead of idling the GPU.
    int32_t cap = 0;
    if (B > 0 && mel_buf && audio_buf) {
        const size_t c1 = mel_cap / ((size_t)B * m->cfg.mel_channels), c2 = audio_cap / ((size_t)B * 64);
        cap = (int32_t)std::min<size_t>(std::min(c1, c2), (size_t)kMaxFrames);
        if (cap > 0 && m2_inference_workspace_bytes(m, B, S, cap) > workspace_bytes) cap = 0;
    }
    const bool spec = cap > 0 && S > 0 && dev_back_ok(m, cap);
    int32_t rc, tmax = 0;
    FrontBufs f;
    if (!spec) {
        if ((rc = m2_inference_front(m, ids, lengths, B, S, scale, front, front_bytes, workspace, workspace_bytes,
                                     &tmax, stream)))
            return rc;
    } else {
        int dev = 0;
        if ((rc = stream_device(st, &dev))) return rc;
        std::lock_guard<std::mutex> lk(g_mb_mu);
        LrMailbox* mb = nullptr;
        if ((rc = mailbox_for(dev, st, &mb))) return rc;
        mb->seq = mb->seq == INT_MAX ? 1 : mb->seq + 1;
        const int32_t seq = mb->seq;
        const CountFuse cf{scale, nullptr, mb->ticket, mb->dev, seq};
        if ((rc = front_run(m, ids, lengths, B, S, front, front_bytes, workspace, workspace_bytes, st, &f,
                            [&](FrontBufs& fb) {
                                return launch_lr_count_sync(fb.dur, 0, scale, B, S, fb.cum, fb.tot, fb.tmax, mb->ticket,
                                                            mb->dev, seq, st);
                            }, &cf)))
            return rc;
        if ((rc = back_run(m, B, S, cap, f.tmax, front, front_bytes, mel_buf, audio_buf, workspace, workspace_bytes,
                           stream)))
            return rc;
        if ((rc = mailbox_wait(mb, seq, st, &tmax, "m2_inference"))) return rc;
        M2_CHECK_SHAPE(tmax <= kMaxFrames, "length regulator: an utterance's frame count exceeds 2^24 (the "
                                           "durations times duration_scale are out of range)");
    }
    const int32_t T = std::max(1, tmax);  // tts_model.py:158-160
    *host_T = T;
    if (spec) {  // done unless T outgrew the capacity (then the launches did nothing)
        *launched = T <= cap ? 1 : 0;
        return M2_OK;
    }
    const size_t need_mel = (size_t)B * T * m->cfg.mel_channels, need_audio = (size_t)B * 64 * T;
    if (!mel_buf || !audio_buf || need_mel > mel_cap || need_audio > audio_cap ||
        m2_inference_workspace_bytes(m, B, S, T) > workspace_bytes)
        return M2_OK;  // the caller allocates for T and calls m2_inference_back
    if ((rc = m2_inference_back(m, B, S, T, front, front_bytes, mel_buf, audio_buf, workspace, workspace_bytes,
                                stream)))
        return rc;
    *launched = 1;
    return M2_OK;
}

size_t m2_inference_workspace_bytes(const m2_model* model, int32_t B, int32_t S, int32_t T) {
    if (!model || B < 0 || S < 0 || T < 0) return 0;
    const int H = model->cfg.hidden_dim;
    Sizer a, b, d;
    carve_tf(a, B, S, H, model->cfg.num_heads, nullptr);
    carve_tf(b, B, T, H, model->cfg.num_heads, nullptr);
    d.off = std::max(b.off, vocoder_ws_bytes(model, B, T));
    (void)d.take<float>((size_t)B * T * H);
    return std::max(a.off, d.off) + 256;
}

int32_t m2_vocoder_path(const m2_model* m) {
    if (!m) return -1;
    return m->x3 ? 2 : (m->fused ? 1 : 0);
}

int32_t m2_transformer_path(const m2_model* m) {
    if (!m) return -1;
    if (!(m->tfused && !m->att_f32)) return 0;
    for (const auto* st : {&m->enc, &m->dec})
        for (const m2_layer_w& L : *st)
            if (L.wide_scores) return 2;
    return 1;
}

int32_t m2_profile_enable(m2_model* m, int32_t capacity) {
    M2_CHECK_ARG(m && capacity >= 0, "m2_profile_enable: bad argument");
    m2_profile_disable(m);
    for (int i = 0; i < capacity * kVocKernels; ++i) {
        hipEvent_t a, b;
        // No system-scope fence: a default event writes back and invalidates
        // L2 at every record, which costs the next kernel its warm weights.
        M2_HIP(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
        M2_HIP(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
        m->prof_begin.push_back(a);
        m->prof_end.push_back(b);
    }
    m->prof_calls = 0;
    m->prof_seen = 0;
    return M2_OK;
}

int32_t m2_profile_read(m2_model* m, float* ms_out, int32_t capacity, int32_t* n_out) {
    M2_CHECK_ARG(m && ms_out && n_out, "m2_profile_read: bad argument");
    const int n = std::min<int>(capacity, m->prof_calls * kVocKernels);
    for (int i = 0; i < n; ++i) {
        ms_out[i] = -1.f;  // kernel not selected
        if (!((m->prof_mask >> (i % kVocKernels)) & 1u)) continue;
        M2_HIP(hipEventSynchronize(m->prof_end[i]));
        M2_HIP(hipEventElapsedTime(&ms_out[i], m->prof_begin[i], m->prof_end[i]));
    }
    *n_out = n;
    m->prof_calls = 0;
    return M2_OK;
}

int32_t m2_profile_select(m2_model* m, uint32_t kernel_mask) {
    M2_CHECK_ARG(m, "m2_profile_select: null model");
    m->prof_mask = kernel_mask;
    return M2_OK;
}

int32_t m2_profile_stride(m2_model* m, int32_t stride) {
    M2_CHECK_ARG(m && stride >= 1, "m2_profile_stride: bad argument");
    m->prof_stride = stride;
    m->prof_seen = 0;
    return M2_OK;
}

int32_t m2_profile_disable(m2_model* m) {
    if (!m) return M2_OK;
    for (auto e : m->prof_begin) (void)hipEventDestroy(e);
    for (auto e : m->prof_end) (void)hipEventDestroy(e);
    m->prof_begin.clear();
    m->prof_end.clear();
    m->prof_calls = 0;
    return M2_OK;
}

}  // extern "C"
