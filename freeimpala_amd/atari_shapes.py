"""Algorithmic work per launch of the Atari-net kernels.

FLOPs count only the dense conv / GEMM arithmetic of each layer (2 * MACs); the zero taps
of the parity-class dgrad formulation and the padded heads columns are NOT counted, so the
roofline fraction is honest. N = (T+1)*B frames per step.
"""


def atari_kernel_work(T: int, B: int, A: int) -> dict:
    N = (T + 1) * B
    O = A + 1
    c1 = 2 * N * 400 * 32 * 256
    c2 = 2 * N * 81 * 64 * 512
    c3 = 2 * N * 49 * 64 * 576
    fc = 2 * N * 512 * 3136
    hd = 2 * N * O * 512
    return {
        "conv1_fwd": ("flop", c1), "conv2_fwd": ("flop", c2), "conv3_fwd": ("flop", c3),
        "fc_fwd": ("flop", fc), "heads_fwd": ("flop", hd),
        "heads_wgrad": ("flop", hd), "heads_dgrad": ("flop", hd),
        "fc_wgrad": ("flop", fc), "fc_dgrad": ("flop", fc),
        "conv3_wgrad": ("flop", c3), "conv3_dgrad": ("flop", c3),
        "conv2_wgrad": ("flop", c2), "conv2_dgrad": ("flop", c2),
        "conv1_wgrad": ("flop", c1),
        # fused frame-resident backward kernels: wgrad + dgrad of the layer in one launch
        "conv2_bwd": ("flop", 2 * c2), "conv3_bwd": ("flop", 2 * c3),
    }


def atari_step_flops(T: int, B: int, A: int) -> int:
    w = atari_kernel_work(T, B, A)
    return sum(v for k, (_, v) in w.items() if not k.endswith("_bwd"))
