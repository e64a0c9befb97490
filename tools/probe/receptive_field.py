"""Receptive field of the SimpleVocoder (reference tts_model.py:243-297) in mel
frames: propagate the index interval of one frame's 64 audio samples back
through output_conv (k3), the ResBlocks (two k3 convs each, components.py:
196-200) and the ConvTranspose1d(k=2r, s=r, p=r/2) upsamplers to the mel
input.  The streamed vocoder's halo (m2_vocoder_halo_frames) must cover it.

    python tools/probe/receptive_field.py  ->  3 3
"""
import math

RATES = (4, 4, 2, 2)


def convT_inputs(a: int, b: int, r: int):
    """Input positions i read by outputs o in [a, b]: o = r*i - r/2 + k, 0 <= k < 2r."""
    p, K = r // 2, 2 * r
    return math.ceil((a + p - (K - 1)) / r), (b + p) // r


def mel_frames_for_samples(a: int, b: int):
    a, b = a - 1, b + 1                      # output_conv k3, padding 1
    for r in reversed(RATES):
        a, b = a - 2, b + 2                  # ResBlock: conv1, conv2 (k3, dilation 1)
        a, b = convT_inputs(a, b, r)         # ConvT upsampler
    return a - 1, b + 1                      # input_conv k3


def halo_frames(frames: int = 16):
    left = right = 0
    for f in range(frames):
        lo, hi = mel_frames_for_samples(64 * f, 64 * f + 63)
        left, right = max(left, f - lo), max(right, hi - f)
    return left, right


if __name__ == "__main__":
    print(*halo_frames())
