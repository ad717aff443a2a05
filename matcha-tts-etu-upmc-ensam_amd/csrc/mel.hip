// Log-mel projection of the data path on gfx950 (reference: matcha/utils/audio_process.py:54-72,
// MelSpectrogram._apply_stft magnitude + __call__'s mel matmul + spectral_normalize_torch).
//
// The STFT itself is torch.stft (rocFFT).  This kernel fuses what follows it -- the magnitude
// sqrt(re^2 + im^2 + 1e-9), the [n_mels x n_freq] mel projection and log(clamp(., 1e-5)) -- into one
// pass over the complex spectrum: the [B, n_freq, F] magnitude tensor and the matmul output never
// reach HBM.  The slaney basis is band-sparse (each bin feeds at most two filters), so each output
// walks only its filter's nonzero bins: ~2 * n_freq multiply-adds per frame instead of
// n_mels * n_freq.  HBM-bound: 8 B per (bin, frame) read once (the other filter's re-read hits L2)
// + 4 B per (mel, frame) written.
//
// Layout: block (64 frames, 4 mels); lanes of a wave are consecutive frames, so every spectrum read
// (one float2 per lane at fixed bin) is a 512-byte coalesced segment and the filter weight is
// wave-uniform (scalar load).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mtts_common.h"

namespace {

constexpr int kMelFrames = 64;
constexpr int kMelRows = 4;

__global__ __launch_bounds__(kMelFrames *kMelRows) void mel_log_kernel(
    const float2 *__restrict__ spec, const float *__restrict__ mel_w, const int32_t *__restrict__ band_lo,
    const int32_t *__restrict__ band_hi, int n_freq, int F, int n_mels, float clip_val, float *__restrict__ out) {
    const int f = blockIdx.x * kMelFrames + threadIdx.x;
    const int m = blockIdx.y * kMelRows + threadIdx.y;
    const int b = blockIdx.z;
    if (m >= n_mels) return;  // wave-uniform (threadIdx.y is constant within a wave)
    const int fc = min(f, F - 1);
    const float2 *s = spec + (size_t)b * n_freq * F + fc;
    const float *w = mel_w + (size_t)m * n_freq;
    const int lo = band_lo[m], hi = band_hi[m];
    float acc = 0.f;
    for (int k = lo; k < hi; ++k) {
        const float2 v = s[(size_t)k * F];
        const float mag = sqrtf(v.x * v.x + v.y * v.y + 1e-9f);
        acc = fmaf(w[k], mag, acc);
    }
    if (f < F) out[((size_t)b * n_mels + m) * F + f] = logf(fmaxf(acc, clip_val));
}

}  // namespace

extern "C" int mtts_mel_log_fwd(const float *spec, const float *mel_w, const int32_t *band_lo, const int32_t *band_hi,
                                int32_t B, int32_t n_freq, int32_t F, int32_t n_mels, float clip_val, float *out,
                                void *hip_stream) {
    MTTS_CHECK_ARG(spec && mel_w && band_lo && band_hi && out, "mel_log_fwd: null pointer");
    MTTS_CHECK_ARG(B >= 0 && n_freq >= 1 && F >= 0 && n_mels >= 1 && B <= 65535 && clip_val > 0.f,
                   "mel_log_fwd: bad shape or clip_val");
    MTTS_CHECK_ARG((uintptr_t)spec % 8 == 0, "mel_log_fwd: spec must be 8-byte aligned (complex64)");
    if ((size_t)B * F == 0) return MTTS_OK;
    dim3 grid((unsigned)((F + kMelFrames - 1) / kMelFrames), (unsigned)((n_mels + kMelRows - 1) / kMelRows), B);
    hipLaunchKernelGGL(mel_log_kernel, grid, dim3(kMelFrames, kMelRows), 0, static_cast<hipStream_t>(hip_stream),
                       reinterpret_cast<const float2 *>(spec), mel_w, band_lo, band_hi, n_freq, F, n_mels, clip_val,
                       out);
    return mtts::check_launch("mel_log_kernel");
}
