/*
 * m2tts_hip.h - C ABI of the MI355X (gfx950) implementation of the m2-tts
 * mel-synthesis + vocoder forward path.
 *
 * The reference (Ryannasr11/m2-tts) has no FFI layer: its boundary is the
 * Python nn.Module API of src/models/tts_model.py and components.py.  Each
 * entry point below replaces the PyTorch op sequence of one reference
 * module's forward; the citation is given per function.  The Python drop-in
 * (m2-tts_amd/src/models/) binds these with ctypes - see INTEGRATION.md.
 *
 * Conventions
 *  - All tensors are caller-owned DEVICE pointers (torch tensor.data_ptr()),
 *    contiguous, fp32 unless stated; ids/lengths are int64.
 *  - `stream` is a hipStream_t passed as void* (torch current stream's
 *    cuda_stream); every call is stream-ordered and asynchronous.  No call
 *    allocates or synchronises, except m2_model_create (one-time weight
 *    packing) and m2_model_destroy.
 *  - Scratch memory is the caller's: size it with m2_workspace_bytes().
 *  - Return 0 on success; M2_E_* (<0) for argument/shape errors; a positive
 *    value is a hipError_t passed through.  m2_last_error() returns a
 *    thread-local message for the last failure on the calling thread.
 *  - One stream per model handle: a model's calls must be ordered on one
 *    stream (or externally synchronised).  The handle carries per-model
 *    device state that successive calls hand over in stream order - the
 *    split-f16 range flag (m2_model_check) and the work-queue counters of the
 *    one-launch transformer layers - so two streams using one handle at the
 *    same time may see each other's range flag and must not share it; create
 *    one handle per stream instead (weights are packed per handle).
 */
#ifndef M2TTS_HIP_H
#define M2TTS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M2_ABI_VERSION 1

#define M2_OK 0
#define M2_E_ARG (-1)         /* null pointer / bad enum / bad size           */
#define M2_E_SHAPE (-2)       /* shape outside what the kernels support       */
#define M2_E_WORKSPACE (-3)   /* workspace smaller than m2_workspace_bytes()  */
#define M2_E_WEIGHTS (-4)     /* weight table incomplete                      */
#define M2_E_INTERNAL (-5)    /* internal protocol failure (see m2_last_error) */
#define M2_E_RANGE (-6)       /* an earlier vocoder call on this model produced non-finite audio
                                 on the split-f16 path (input or activation outside its range);
                                 see m2_model_check / m2_set_range_policy                        */

/* M2TTSModel.__init__ hyper-parameters (tts_model.py:303-313), plus the
 * positional-encoding table length (TextEncoder max_seq_len, tts_model.py:29). */
typedef struct m2_config {
    int32_t vocab_size;          /* 256 */
    int32_t hidden_dim;          /* H: 64 stage1, 96 stage2 */
    int32_t mel_channels;        /* M: 64 / 80 */
    int32_t text_encoder_layers; /* 2 / 3 */
    int32_t decoder_layers;      /* 2 / 3 */
    int32_t num_heads;           /* 2 */
    int32_t vocoder_channels;    /* C: 128 / 256 */
    int32_t max_positions;       /* 1000 */
} m2_config;

typedef struct m2_model m2_model;

int32_t m2_abi_version(void);
const char* m2_last_error(void);

/* ---- weight table ---------------------------------------------------------
 * The weights are addressed by their reference state_dict key
 * (M2TTSModel.state_dict(), tts_model.py:303-343).  m2_weight_count/name/numel
 * enumerate the keys in the order m2_model_create expects. */
int32_t m2_weight_count(const m2_config* cfg);
int32_t m2_weight_name(const m2_config* cfg, int32_t index, char* buf, int32_t buflen);
int64_t m2_weight_numel(const m2_config* cfg, int32_t index);

/* Packs and uploads the weights once (BatchNorm folded into the duration
 * convs, conv weights re-laid out for the kernels).  `weights[i]` is a device
 * pointer to the tensor named by m2_weight_name(cfg, i) (fp32; the BatchNorm
 * num_batches_tracked entries are int64 and ignored).  Synchronises `stream`. */
int32_t m2_model_create(const m2_config* cfg, const void* const* weights, int32_t n_weights,
                        void* stream, m2_model** out);
int32_t m2_model_destroy(m2_model* model);

/* Re-reads the developer switches (M2_* environment variables that force one
 * code path for A/B comparisons and tests) into the library's switch table.
 * The table is read when the library loads and at every m2_model_create;
 * no entry point reads the environment per call.  Not part of the
 * reference's surface (it has no FFI). */
void m2_reload_switches(void);
int32_t m2_model_config(const m2_model* model, m2_config* out);

/* Scratch bytes needed by the stage calls for a batch of B utterances of S
 * phonemes and T mel frames (T = 0: encoder/duration only). */
size_t m2_workspace_bytes(const m2_model* model, int32_t B, int32_t S, int32_t T);

/* ---- stage entry points ---------------------------------------------------*/

/* TextEncoder.forward (tts_model.py:57-89): embedding*sqrt(H) + pe, L_enc pre-LN
 * transformer layers with key-padding mask (components.py:131-140, 59-90,
 * 226-241), final LayerNorm.  lengths may be NULL (no mask).
 * out_enc [B,S,H]; out_mask [B,S] uint8 (may be NULL). */
int32_t m2_text_encoder(const m2_model* model, const int64_t* ids, const int64_t* lengths,
                        int32_t B, int32_t S, float* out_enc, uint8_t* out_mask,
                        void* workspace, size_t workspace_bytes, void* stream);

/* DurationPredictor.forward (tts_model.py:99-117): 2x[Conv1d k3 + BN(eval) +
 * ReLU] -> Conv1d k1 -> softplus.  enc [B,S,H] -> out_dur [B,S]. */
int32_t m2_duration_predictor(const m2_model* model, const float* enc, int32_t B, int32_t S,
                              float* out_dur, void* workspace, size_t workspace_bytes, void* stream);

/* LengthRegulator.forward, counting half (tts_model.py:146-162): per phoneme
 * n = int(trunc(dur*scale)) (fp32 product, truncation toward zero, n<=0 -> 0);
 * per utterance exclusive prefix sums out_cum [B,S+1] (int32), totals
 * out_T [B] and the batch maximum out_Tmax [1] (int32).  `dur` is fp32, or
 * int32 when dur_is_int != 0 (scale then ignored). */
int32_t m2_length_regulator_count(const void* dur, int32_t dur_is_int, float scale,
                                  int32_t B, int32_t S, int32_t* out_cum, int32_t* out_T,
                                  int32_t* out_Tmax, void* stream);

/* m2_length_regulator_count, plus the one host read the regulator needs
 * (tts_model.py:163-166: the batch maximum sizes the output): also stores
 * T_max into *host_Tmax (host memory) before returning, by a mailbox the
 * count kernel posts to coherent host-mapped memory, polled by this call -
 * in place of a device->host copy and a stream synchronisation.  Blocks the
 * calling thread until the work queued on `stream` before it and the count
 * kernel are done.  One calling thread per device. */
int32_t m2_length_regulator_count_sync(const void* dur, int32_t dur_is_int, float scale,
                                       int32_t B, int32_t S, int32_t* out_cum, int32_t* out_T,
                                       int32_t* out_Tmax, int32_t* host_Tmax, void* stream);

/* LengthRegulator.forward, expanding half (tts_model.py:146-178): frame t of
 * utterance b copies enc[b, s] for cum[b,s] <= t < cum[b,s+1]; frames past
 * the utterance's total are zero; the output has exactly T_out frames
 * (padding or truncation, tts_model.py:165-176).  out [B,T_out,H]. */
int32_t m2_length_regulator_expand(const float* enc, const int32_t* cum, int32_t B, int32_t S,
                                   int32_t H, int32_t T_out, float* out, void* stream);

/* MelDecoder.forward (tts_model.py:211-228): L_dec pre-LN transformer layers
 * WITHOUT mask over the frames, LayerNorm, Linear(H->M).
 * x [B,T,H] -> out_mel [B,T,M].  x is not modified. */
int32_t m2_mel_decoder(const m2_model* model, const float* x, int32_t B, int32_t T, float* out_mel,
                       void* workspace, size_t workspace_bytes, void* stream);

/* SimpleVocoder.forward (tts_model.py:279-297): input_conv, 4x[ConvT(k=2r,s=r,
 * p=r/2) + leaky(0.1) + LightweightResBlock], output_conv + tanh.
 * mel_layout 0: mel [B,M,T] (the module's own input); 1: mel [B,T,M] (the
 * decoder output, read transposed in place).  out_audio [B,1,64T]. */
int32_t m2_vocoder(const m2_model* model, const float* mel, int32_t mel_layout, int32_t B,
                   int32_t T, float* out_audio, void* workspace, size_t workspace_bytes,
                   void* stream);

/* ---- streamed / chunked vocoder (long-form; SURVEY 8b `chunk_frames`) ------
 * The reference runs SimpleVocoder over the whole mel (tts_model.py:279-297).
 * A chunk [f0, f1) of mel frames is computed over the window
 * [f0 - halo, f1 + halo) clipped to [0, T), halo = m2_vocoder_halo_frames()
 * = the vocoder's receptive field (3 frames per side), so every audio sample
 * equals the whole-utterance call's bit for bit; the window's mel is copied to
 * the workspace, vocoded, and the centre of its audio copied out.
 *   m2_vocoder_set_chunking: m2_vocoder (and m2_inference / _back) then run
 *     chunk_frames frames at a time (0 = whole utterance, the default); size
 *     the workspace after changing it (m2_workspace_bytes depends on it).
 *   m2_vocoder_chunk: audio of frames [f0, f1) only, out_chunk [B,1,64(f1-f0)]
 *     (for streaming: chunk k can be played while chunk k+1 is computed);
 *     workspace from m2_vocoder_chunk_workspace_bytes(B, T, f1 - f0). */
int32_t m2_vocoder_set_chunking(m2_model* model, int32_t chunk_frames);
int32_t m2_vocoder_halo_frames(void);
int32_t m2_vocoder_chunk(const m2_model* model, const float* mel, int32_t mel_layout, int32_t B,
                         int32_t T, int32_t f0, int32_t f1, float* out_chunk, void* workspace,
                         size_t workspace_bytes, void* stream);
size_t m2_vocoder_chunk_workspace_bytes(const m2_model* model, int32_t B, int32_t T,
                                        int32_t chunk_frames);

/* ---- range of the split-f16 arithmetic -------------------------------------
 * The split path carries fp32 values as f16 hi/lo pairs; a value of magnitude
 * >= 65520 (input mel or any activation) becomes hi = inf, lo = NaN, and the
 * NaN reaches the audio, whose last kernel raises a per-model flag (never a
 * silently wrong finite result).  Transformer activations are bounded by the
 * LayerNorm weights and checked once at m2_model_create (out of range -> the
 * exact-f32 transformer kernels).  What a raised flag does:
 *   policy 0 (report, default): asynchronous, like a HIP kernel error - the
 *     next m2_vocoder / m2_inference* call on the model returns M2_E_RANGE
 *     (and clears the flag); m2_model_check synchronises `stream` and
 *     reports it at once (*flagged = 1, flag cleared).
 *   policy 1 (fallback): the non-finite part of the call is recomputed in
 *     fp32 on the device, without a host wait.  On the pipelined tails (the
 *     stage1 / stage2 split-f16 defaults) each workgroup whose strip stored a
 *     non-finite sample recomputes only that strip's frames inside the tail
 *     launch by direct fp32 convolution in the reference's layer order
 *     (csrc/vocoder_redo.h): the reference's op sequence in fp32, in another
 *     summation order than the exact-f32 kernels, so within the
 *     reference-conditioned tolerance of tests/test_gpu_range.py, NOT
 *     bit-equal to them; non-finite only if the reference's result is.
 *     M2_REDO_LAUNCH=1 (and the windowed x3 tails) instead enqueue the
 *     guarded exact-f32 launch behind the split kernels (it returns at once
 *     unless their device flag word is raised; two words alternate between
 *     calls, the next call's first kernel zeroes the other), whose output is
 *     bit-equal to the exact-f32 kernels.  Other shapes: m2_vocoder
 *     synchronises `stream` and re-runs the call on the exact-f32 kernels. */
int32_t m2_set_range_policy(m2_model* model, int32_t policy);
int32_t m2_model_check(m2_model* model, void* stream, int32_t* flagged);

/* Select the vocoder arithmetic at run time: 1 = exact-f32 MFMA kernels,
 * 2 = split-f16 MFMA kernels (the default when the model has their packs).
 * M2_E_ARG when the model has no packs for the requested path. */
int32_t m2_vocoder_select(m2_model* model, int32_t path);

/* ---- whole-inference entry points (M2TTSModel.inference, tts_model.py:402-438)
 * Two calls split at the one host read the path needs (T_max sizes the
 * outputs), so a step costs two host->library crossings instead of six:
 *   m2_inference_front: text encoder (+ padding mask when lengths != NULL),
 *     duration predictor, frame counts; blocks until T_max is posted
 *     (as m2_length_regulator_count_sync) and stores it in *host_Tmax.
 *   m2_inference_back: length-regulator expansion to T frames (the caller
 *     passes max(1, T_max), tts_model.py:158-160), mel decoder, vocoder.
 *     out_mel [B,T,M], out_audio [B,1,64T].
 * `front` (m2_front_bytes(B,S)) carries the encoder output, durations and
 * frame counts from the first call to the second; `workspace` is sized by
 * m2_inference_workspace_bytes(B,S,T) (T = 0 for the front call). */
size_t m2_front_bytes(const m2_model* model, int32_t B, int32_t S);
size_t m2_inference_workspace_bytes(const m2_model* model, int32_t B, int32_t S, int32_t T);
int32_t m2_inference_front(const m2_model* model, const int64_t* ids, const int64_t* lengths,
                           int32_t B, int32_t S, float scale, void* front, size_t front_bytes,
                           void* workspace, size_t workspace_bytes, int32_t* host_Tmax,
                           void* stream);
int32_t m2_inference_back(const m2_model* model, int32_t B, int32_t S, int32_t T,
                          const void* front, size_t front_bytes, float* out_mel,
                          float* out_audio, void* workspace, size_t workspace_bytes,
                          void* stream);

/* Both halves in ONE call when the outputs fit.  The buffers give a frame
 * capacity T_cap = min(mel_cap / (B*M), audio_cap / (B*64)) (if the workspace
 * holds m2_inference_workspace_bytes(B,S,T_cap)); with one, and when
 * m2_inference_dev_supported(model, T_cap), the back half is enqueued right
 * behind the count kernel BEFORE the host reads T_max, its grids sized for
 * T_cap and its kernels taking T = max(1, T_max) from the device (the host
 * wait then overlaps the decoder instead of idling the GPU); otherwise it is
 * enqueued after the read, if B*T*M / B*64*T fit.  The outputs are written
 * contiguously from the start of the buffers ([B,T,M] and [B,1,64T]) and
 * *launched = 1.  When T exceeds the capacity (the speculative launches then
 * did nothing) *launched = 0 and the caller allocates for *host_T and calls
 * m2_inference_back (the front buffer holds the hand-off).
 * M2_SPECULATIVE=0 in the environment turns the device-side frame count off. */
int32_t m2_inference(const m2_model* model, const int64_t* ids, const int64_t* lengths, int32_t B,
                     int32_t S, float scale, void* front, size_t front_bytes, void* workspace,
                     size_t workspace_bytes, float* mel_buf, size_t mel_cap, float* audio_buf,
                     size_t audio_cap, int32_t* host_T, int32_t* launched, void* stream);

/* Device-side frame count for sharded inference (no host read between the
 * halves): m2_inference_front_dev writes this shard's T_max to the device word
 * dev_Tmax (e.g. the payload of the ranks' all-reduce(MAX)) without waiting;
 * m2_inference_back_dev launches the back half for a capacity of T_cap frames
 * and takes T = max(1, *dev_T) from the device; when T > T_cap it does
 * nothing (the caller reads T and runs m2_inference_back).  Outputs as
 * m2_inference's.  m2_inference_dev_supported: 1 when this model's back half
 * can run so at T_cap (one-launch decoder layers with the fused mel
 * projection, the fused unchunked vocoder).  The back half's first launch
 * posts T = max(1, *dev_T) (also when it exceeds T_cap) to a host-mapped word
 * of the model: m2_frames_wait blocks until the post of the model's latest
 * m2_inference_back_dev call is visible and returns that T (no stream
 * synchronisation, no copy: the back half keeps running). */
int32_t m2_inference_dev_supported(const m2_model* model, int32_t T_cap);
int32_t m2_inference_front_dev(const m2_model* model, const int64_t* ids, const int64_t* lengths,
                               int32_t B, int32_t S, float scale, void* front, size_t front_bytes,
                               void* workspace, size_t workspace_bytes, int32_t* dev_Tmax, void* stream);
int32_t m2_inference_back_dev(const m2_model* model, int32_t B, int32_t S, int32_t T_cap,
                              const int32_t* dev_T, const void* front, size_t front_bytes,
                              float* out_mel, float* out_audio, void* workspace,
                              size_t workspace_bytes, void* stream);
int32_t m2_frames_wait(const m2_model* model, void* stream, int32_t* host_T);

/* ---- kernel-level entry points (for the components API and tests) ---------*/

/* LightweightResBlock.forward (components.py:196-200) of vocoder stage k
 * (0..3): y = conv2(leaky(conv1(x))) + x.  x,y [B,c_k,L]; tmp: B*c_k*L floats. */
int32_t m2_vocoder_resblock(const m2_model* model, int32_t k, const float* x, int32_t B, int32_t L,
                            float* y, float* tmp, void* stream);

/* leaky(ConvTranspose1d) of vocoder stage k (tts_model.py:255-263, 291):
 * x [B,c,L] -> y [B,c/2,r*L]. */
int32_t m2_vocoder_upsample(const m2_model* model, int32_t k, const float* x, int32_t B, int32_t L,
                            float* y, void* stream);

/* Standalone kernels with caller-supplied weights in PyTorch layout (used by
 * the components API for modules that live outside an M2TTSModel). */

/* y = act((conv1d(x; w [Cout,Cin,ksize], b [Cout], padding ksize/2) [* alpha + beta]))
 * (+ res).  ksize 1 or 3; alpha/beta per output channel (the BatchNorm1d eval
 * form, components.py:170-171) or NULL; act 0 none, 1 leaky(0.1), 2 tanh,
 * 3 relu, 4 softplus(beta=1, threshold=20).  x [B,Cin,L], y/res [B,Cout,L].
 * Serves Conv1d in ConvBlock, VariancePredictor.projection, the vocoder's
 * input/output convs and LightweightResBlock convs used outside a model. */
int32_t m2_conv1d(const float* x, const float* w, const float* b, const float* alpha,
                  const float* beta, const float* res, int32_t ksize, int32_t act, int32_t B,
                  int32_t Cin, int32_t Cout, int32_t L, float* y, void* stream);

/* m2_conv1d for any kernel size, dilation and zero padding (components.py:
 * 143-200 ConvBlock(kernel_size), LightweightResBlock(kernel_size, dilation),
 * tts_model.py:246,272 SimpleVocoder(kernel_size)): y [B,Cout,Lo] with
 * Lo = L + 2*padding - dilation*(ksize-1); res (optional) needs Lo == L. */
int32_t m2_conv1d_ex(const float* x, const float* w, const float* b, const float* alpha, const float* beta,
                     const float* res, int32_t ksize, int32_t dilation, int32_t padding, int32_t act, int32_t B,
                     int32_t Cin, int32_t Cout, int32_t L, float* y, void* stream);

/* y = act(convT1d(x; w [Cin,Cout,2r], b, stride r, padding r/2)), r in {2,4};
 * x [B,Cin,L] -> y [B,Cout,r*L] (tts_model.py:255-263, 291). */
int32_t m2_conv_transpose1d(const float* x, const float* w, const float* b, int32_t rate,
                            int32_t act, int32_t B, int32_t Cin, int32_t Cout, int32_t L, float* y,
                            void* stream);

/* y[R,N] = act(LN?(x)[R,K] . w[N,K]^T + b) (+ res[R,N]).  gamma/beta NULL:
 * no LayerNorm (eps 1e-5); b may be NULL; act 0 none, 3 relu. */
int32_t m2_linear(const float* x, const float* gamma, const float* beta, const float* w,
                  const float* b, const float* res, int32_t act, int32_t R, int32_t K, int32_t N,
                  float* y, void* stream);

/* y[R,K] = LN(x) with affine gamma/beta, eps 1e-5. */
int32_t m2_layer_norm(const float* x, const float* gamma, const float* beta, int32_t R, int32_t K,
                      float* y, void* stream);

/* Attention core of MultiHeadAttention.forward (components.py:72-86):
 * qkv [B,N,3H] laid out (3, heads, hd) per row as the reference's reshape
 * implies; key_mask [B,N] uint8 or NULL (masked keys score -1e9);
 * out [B,N,H] (heads re-interleaved, before out_proj).  head_dim 16/32/48/64
 * run on the MFMA kernels, any other head_dim <= 256 on a generic fp32 one. */
int32_t m2_attention(const float* qkv, const uint8_t* key_mask, int32_t B, int32_t N, int32_t H,
                     int32_t heads, float* out, void* stream);

/* TextEncoder embedding (tts_model.py:78-80): y[b,s,:] = emb[ids[b,s],:] *
 * scale + pe[s,:] (scale = sqrt(H) as fp32); ids outside [0,vocab) read zeros. */
int32_t m2_embed_positional(const int64_t* ids, const float* emb, const float* pe, int32_t B,
                            int32_t S, int32_t H, int32_t vocab, float scale, float* y,
                            void* stream);

/* PositionalEncoding.forward (components.py:30-39): y = x + pe[:S] (x [B,S,H]). */
int32_t m2_add_positional(const float* x, const float* pe, int32_t B, int32_t S, int32_t H,
                          float* y, void* stream);

/* ---- mel features and Griffin-Lim (src/utils/audio.py:45-151) --
 * The reference's librosa calls: compute_mel_spectrogram = melspectrogram
 * (periodic Hann, centre zero padding, Slaney mel filters, power 2) ->
 * power_to_db(ref=max, amin 1e-10, top_db 80) -> [-1, 1] normalisation, per
 * utterance; mel_to_audio = (x+1)/2 -> db_to_power -> NNLS against the mel
 * filters (mel_to_stft; here Nesterov projected gradient from the clipped
 * pseudo-inverse - librosa uses scipy L-BFGS-B from the same start) -> sqrt
 * -> griffinlim(n_iter, momentum) -> istft -> / max|y|.
 *   m2_dsp_create: the tables (window, twiddles, mel filters, pseudo-inverse)
 *     for one (sr, n_fft in {512, 1024, 2048}, hop, win_length, n_mels, fmin,
 *     fmax); synchronises `stream`.
 *   audio [B, L] fp32; frames T = m2_dsp_frames(L) = 1 + L / hop;
 *   m2_stft -> complex64 [B, T, n_fft/2 + 1]; m2_mel_spectrogram -> out_mel
 *     [B, n_mels, T] normalised dB;
 *   m2_griffin_lim: from mel [B, n_mels, T] (normalised dB; magnitudes as
 *     m2_mel_to_magnitude) or, when mag != NULL, from magnitudes
 *     [B, T, n_fft/2+1] (bare griffinlim, no peak normalisation);
 *     init_angles complex64 [B, T, n_fft/2+1] unit phases (librosa's
 *     init='random' draw, made explicit); out_audio [B, hop (T - 1)]. */
typedef struct m2_dsp m2_dsp;
int32_t m2_dsp_create(int32_t sample_rate, int32_t n_fft, int32_t hop_length, int32_t win_length,
                      int32_t n_mels, float fmin, float fmax, void* stream, m2_dsp** out);
int32_t m2_dsp_destroy(m2_dsp* dsp);
int32_t m2_dsp_frames(const m2_dsp* dsp, int32_t L);
int32_t m2_stft(const m2_dsp* dsp, const float* audio, int32_t B, int32_t L, void* out_spec, void* stream);
int32_t m2_mel_spectrogram(const m2_dsp* dsp, const float* audio, int32_t B, int32_t L, float* out_mel,
                           void* stream);
/* mel_to_stft alone (librosa.feature.inverse.mel_to_stft, power 2, as
 * audio.py:138 reaches it): mel [B, n_mels, T] -> magnitudes out_mag
 * [B, T, n_fft/2+1] = sqrt(librosa.util.nnls(mel_basis, db_to_power)).
 * librosa's L-BFGS-B stops at its start X0 = max(0, pinv(W) M) whenever the
 * block's projected gradient there is <= 1e-5 (every mel in the normalised
 * range); that test is made exactly and X0 returned; a block that would
 * iterate gets nnls_iters projected-gradient steps per frame instead.
 * Scratch: m2_mel_to_magnitude_workspace_bytes. */
size_t m2_mel_to_magnitude_workspace_bytes(const m2_dsp* dsp, int32_t B, int32_t T);
int32_t m2_mel_to_magnitude(const m2_dsp* dsp, const float* mel, int32_t B, int32_t T, int32_t nnls_iters,
                            float* out_mag, void* workspace, size_t workspace_bytes, void* stream);
size_t m2_griffin_lim_workspace_bytes(const m2_dsp* dsp, int32_t B, int32_t T);
int32_t m2_griffin_lim(const m2_dsp* dsp, const float* mel, const float* mag, const void* init_angles,
                       int32_t B, int32_t T, int32_t n_iter, float momentum, int32_t nnls_iters,
                       float* out_audio, void* workspace, size_t workspace_bytes, void* stream);

/* ---- measurement ----------------------------------------------------------
 * Kernel timing with HIP events recorded on the launch stream around each of
 * the fused vocoder's kernels (bench.py's roofline).  enable: allocate event
 * pairs for `capacity` m2_vocoder calls (outside any timed region); each call
 * then records one pair per kernel while capacity lasts.  read: synchronise
 * and return durations in ms, call-major ([call][kernel]), n_out = count, and
 * reset.  Kernels are named by m2_profile_kernel_name(i), i < count(). */
int32_t m2_profile_enable(m2_model* model, int32_t capacity);
int32_t m2_profile_read(m2_model* model, float* ms_out, int32_t capacity, int32_t* n_out);
int32_t m2_profile_disable(m2_model* model);
/* Record event pairs only around the kernels whose bit is set (default all);
 * m2_profile_read reports -1 for the others.  Every recorded event costs a
 * few microseconds of pipeline drain between kernels. */
int32_t m2_profile_select(m2_model* model, uint32_t kernel_mask);
/* Record on every `stride`-th m2_vocoder call only (default 1; the calls in
 * between record nothing and take no capacity), so a timed region can carry a
 * sample of the launches at a fraction of the event cost.  Reset by enable. */
int32_t m2_profile_stride(m2_model* model, int32_t stride);
int32_t m2_profile_kernel_count(void);
const char* m2_profile_kernel_name(int32_t index);
/* The same kernel as launched by this model (symbol prefix = rocprofv3 name). */
const char* m2_profile_kernel_name_for(const m2_model* model, int32_t index);
/* Vocoder arithmetic of this model: 0 per-layer fp32 kernels, 1 fused exact-f32
 * MFMA (v_mfma_f32_16x16x4_f32), 2 fused split-f16 MFMA (fp32 operands as
 * f16 hi/lo pairs, 3 products per fp32 product, fp32 accumulation). */
int32_t m2_vocoder_path(const m2_model* model);
/* Transformer arithmetic of this model: 1 = fused split-f16 layers and
 * attention, 2 = the same with at least one layer whose attention-score bound
 * reaches the f16 maximum (that layer keeps its softmax base in fp32 in every
 * attention form), 0 = fp32 linears and the exact-f32 attention (weights
 * whose activation bound leaves the f16 range, or M2_TF_UNFUSED / M2_ATT_F32). */
int32_t m2_transformer_path(const m2_model* model);

#ifdef __cplusplus
}
#endif
#endif /* M2TTS_HIP_H */
