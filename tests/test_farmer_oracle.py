"""The FarmerLstm CPU oracle (oracle/farmer_oracle.py) against the reference's own model:
golden fixtures made by running gpu_benchmark.FarmerLstmModel + its train step
(tests/golden/make_farmer_golden.py). Parity pinned by the reference: value, loss, every
gradient and the parameters after two optimizer steps (adam, adamw, sgd; mse, huber, mae)."""
import numpy as np
import pytest

from farmer_golden import cases, compare_blob, load


def test_param_count_matches_reference_model():
    from oracle import farmer_oracle as fo
    assert fo.PARAM_COUNT == 1_514_497  # SURVEY.md section 6 (gpu_benchmark.py's model)


@pytest.mark.parametrize("path", cases(), ids=lambda p: p.split("/")[-1][:-4])
def test_farmer_oracle_vs_reference_golden(path):
    from oracle import farmer_oracle as fo
    g = load(path)
    p = fo.gen_params(int(g["param_seed"]))
    opt = fo.Optimizer(str(g["optimizer"]), float(g["lr"]), fo.PARAM_COUNT)
    offs = fo.offsets()
    for s in range(int(g["steps"])):
        val, lv, grad, p = fo.train_step(p, opt, g["z"], g["x"], g["y"], str(g["loss_kind"]))
        np.testing.assert_allclose(val, g[f"step{s}/value"], rtol=1e-5, atol=1e-6)
        assert abs(lv - float(g[f"step{s}/loss"])) <= 1e-5 * max(1.0, abs(lv))
        compare_blob(g, s, "grad", grad, offs, rtol=1e-4, atol_frac=1e-5, what="oracle grad")
        compare_blob(g, s, "param", p, offs, rtol=1e-6, atol_frac=1e-5, what="oracle param",
                     adam=str(g["optimizer"]) != "sgd")
