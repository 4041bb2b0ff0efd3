"""farmer_probe.py -- repeated FarmerLstm steps vs the fp64 oracle for the recurrence shapes
(R = 1 / 2 / 4 rows per workgroup), printing per repetition the max error of h_T (the LSTM
kernel's output) and of the values. Diagnostic for history-dependent failures."""
import sys
import os
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from freeimpala_amd.farmer import FarmerLstmModel
    from freeimpala_amd import hip
    from oracle import farmer_oracle as fo

    def junk():
        bufs = [hip.DeviceBuffer(64 << 20) for _ in range(4)]
        for j in bufs:
            j.upload(np.full((64 << 20) // 4, np.nan, np.float32))
        hip.synchronize()
        for j in bufs:
            j.free()
    for B, T in ((40, 33), (301, 7), (601, 5), (64, 100)):
        p0 = fo.gen_params(5)
        z, x, y = fo.gen_inputs(6, B, T)
        v_ref, saved = fo.forward(p0, z, x)
        h_ref = saved["acts"][0][:, :128]
        for rep in range(4):
            if rep >= 2:
                junk()
            M = FarmerLstmModel(batch_size=B, seq_length=T, loss="mse", optimizer="sgd", lr=1e-2, params=p0)
            lv, val = M.train_step(z, x, y, with_values=True)
            h = M.tensor_array("h_last", (B, 612))[:, :128]
            g = M.tensor_array("gates", (B, T, 512))
            eh = np.abs(h - h_ref).max()
            ev = np.abs(val.ravel() - v_ref.ravel()).max()
            eg = max(np.abs(g[:, t, :] - np.concatenate([saved["gates"][t][i] for i in range(4)], axis=1)).max()
                     for t in range(T))
            cat = M.tensor_array("h_last", (B, 612))
            ex = np.abs(cat[:, 128:] - x).max()
            acts = [M.tensor_array(f"act{l}", (B, 512)) for l in range(1, 6)]
            ea = [float(np.abs(acts[l - 1] - saved["acts"][l]).max()) for l in range(1, 6)]
            print(f"B={B} T={T} rep={rep}: |h_T| err {eh:.2e} (|h| max {np.abs(h_ref).max():.2e}, gpu h absmax "
                  f"{np.abs(h).max():.2e}) gates err {eg:.2e} cat_x err {ex:.2e} acts err {['%.1e' % e for e in ea]} "
                  f"values err {ev:.2e} nan {int(np.isnan(val).sum())}", flush=True)
            M.close()


if __name__ == "__main__":
    main()
