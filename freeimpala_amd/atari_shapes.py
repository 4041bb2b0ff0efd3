"""Algorithmic work per launch of the Atari-net kernels.

Each kernel site gets (FLOPs, HBM bytes). FLOPs count only the dense conv / GEMM arithmetic
of each layer (2 * MACs); the zero taps of the parity-class dgrad formulation and the padded
heads columns are NOT counted. Bytes count each tensor the kernel must read or write once
(u8 frames, bf16 activations / data-gradients, fp32 weight-gradient partials ignored: they
are < 0.1 % of the traffic). The roofline bound of a kernel is the resource whose time at
peak is larger (MI355X: 2.5 PF/s bf16 MFMA, 8 TB/s HBM). N = (T+1)*B frames per step.
"""

FRAME = 84 * 84 * 4      # u8 bytes per frame
A1 = 20 * 20 * 32 * 2    # bf16 bytes per frame: a1 / da1
A2 = 9 * 9 * 64 * 2      # a2 / da2
A3 = 7 * 7 * 64 * 2      # a3 / da3
H = 512 * 2              # h / dh


def atari_kernel_work(T: int, B: int, A: int) -> dict:
    """tag -> (flops, bytes) per launch."""
    N = (T + 1) * B
    O = A + 1
    c1 = 2 * N * 400 * 32 * 256
    c2 = 2 * N * 81 * 64 * 512
    c3 = 2 * N * 49 * 64 * 576
    fc = 2 * N * 512 * 3136
    hd = 2 * N * O * 512
    return {
        "conv1_fwd": (c1, N * (FRAME + A1)),
        "conv2_fwd": (c2, N * (A1 + A2)),
        "conv3_fwd": (c3, N * (A2 + A3)),
        "fc_fwd": (fc, N * (A3 + H)),
        "heads_fwd": (hd, N * (H + 4 * O)),
        "heads_wgrad": (hd, N * (H + 4 * O)),
        "heads_dgrad": (hd, N * (4 * O + 2 * H)),          # dout in, h mask in, dh out
        "fc_wgrad": (fc, N * (A3 + H)),
        "fc_dgrad": (fc, N * (H + A3)),
        "conv3_wgrad": (c3, N * (A2 + A3)),
        "conv3_dgrad": (c3, N * (2 * A3 + 2 * A2)),
        "conv2_wgrad": (c2, N * (A1 + A2)),
        "conv2_dgrad": (c2, N * (A2 + 2 * A1)),
        "conv1_wgrad": (c1, N * (FRAME + A1)),
        # fused frame-resident backward kernels (wgrad + dgrad + bias of the layer):
        # conv3 reads a2, da3 (unmasked) and its mask a3, writes da2; conv2 reads a1, da2, writes da1
        "conv2_bwd": (2 * c2, N * (A1 + A2 + A1)),
        "conv3_bwd": (2 * c3, N * (A2 + 2 * A3 + A2)),
        # fused conv1 + conv2 forward: frames in, a1 and a2 out (a1 is not read back)
        "conv12_fwd": (c1 + c2, N * (FRAME + A1 + A2)),
        # fused conv2 backward + conv1 weight gradient: a1, da2, frames in (da1 stays in LDS)
        "conv21_bwd": (2 * c2 + c1, N * (A1 + A2 + FRAME)),
    }


def atari_step_flops(T: int, B: int, A: int) -> int:
    w = atari_kernel_work(T, B, A)
    return sum(f for k, (f, _) in w.items() if not k.endswith("_bwd") and k != "conv12_fwd")  # each layer once
