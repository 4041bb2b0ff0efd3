"""LDS bank model checks of the conv3 reshuffle lane order (CPU only).

The conv3 forward / backward kernels move each landed 1-KiB staging piece into their LDS
image with lane L carrying unit rs_lane(L) of the piece (csrc/atari_fr.hip, rs_lane). These
tests re-derive the bank cost of that order with the MI355X_MICROARCH.md lane-group rules
(scripts/lds_conflicts.py) and pin the property the kernels rely on: ds_write_b128 groups
conflict-free for the chunk-planar X image, staging ds_read_b128 groups conflict-free, and
the bordered dY image no worse than 2-way. The rs_lane expression is parsed from the HIP
source, so the test follows the kernel.
"""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("lds_conflicts", os.path.join(ROOT, "scripts", "lds_conflicts.py"))
lds = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(lds)


def _rs_lane():
    src = open(os.path.join(ROOT, "freeimpala_amd", "csrc", "atari_fr.hip")).read()
    m = re.search(r"int rs_lane\(int L\) \{ return ([^;]+); \}", src)
    assert m, "rs_lane not found in atari_fr.hip"
    expr = m.group(1)
    return [eval(expr, {}, {"L": L}) for L in range(64)]


def _zc(c):
    return 8 * (c & 1) + 4 * ((c >> 1) & 1)


def _x_unit(i):  # a2 unit (pixel-major, 8 chunks) -> chunk-planar image unit
    p, c = i >> 3, i & 7
    return p + 96 * c + _zc(c)


def _dy_unit(i):  # da3 unit (pixel-major, 8 chunks) -> bordered 11x11 image unit
    q, c = i >> 3, i & 7
    y, x = q // 7, q % 7
    return 9 * (y + 2) + (x + 2) + 128 * c + _zc(c)


def _write_cycles(units):
    """ds_write_b128: 8 groups of 8 contiguous lanes, bank (a/4) mod 32 (one LDS cycle per
    group when conflict-free)."""
    tot = 0
    for k in range(8):
        banks = {}
        for l in range(8 * k, 8 * k + 8):
            if units[l] is None:
                continue
            for d in range(4):
                dw = 4 * units[l] + d
                banks.setdefault(dw % 32, set()).add(dw)
        tot += max((len(v) for v in banks.values()), default=1)
    return tot


def _piece_costs(order, unit_of, nunits):
    w = r = 0
    for j in range((nunits + 63) // 64):
        units = [unit_of(64 * j + order[L]) if 64 * j + order[L] < nunits else None for L in range(64)]
        w += _write_cycles(units)
        r += lds.cycles([16 * order[L] for L in range(64)], "b128")  # staging read of the piece
    return w, r


def test_rs_lane_is_a_permutation():
    assert sorted(_rs_lane()) == list(range(64))


def test_x_image_reshuffle_is_conflict_free():
    order = _rs_lane()
    pieces = (648 + 63) // 64
    w, r = _piece_costs(order, _x_unit, 648)
    assert w == 8 * pieces and r == 4 * pieces  # one LDS cycle per lane group
    w_id, _ = _piece_costs(list(range(64)), _x_unit, 648)
    assert w_id > 3 * w  # the identity order is 4-way on most groups


def test_dy_image_reshuffle_at_most_two_way():
    order = _rs_lane()
    pieces = (392 + 63) // 64
    w, r = _piece_costs(order, _dy_unit, 392)
    assert r == 4 * pieces
    assert w <= 2 * 8 * pieces
    w_id, _ = _piece_costs(list(range(64)), _dy_unit, 392)
    assert w < w_id
