"""Per-channel gradient error distribution of the engine vs the fp64 oracles
(diagnostic for tests/test_gpu_engine.py::test_bf16_grads_per_channel_vs_rounded_oracle).

    python tools/probes/perchannel_diag.py SPEC_NAME [B] [seed]

Prints, per layer and for bf16 (vs the bf16-rounded oracle) and fp32 (vs the
exact oracle): max / 99th pct / median per-channel relative error, so a
systematic error (every channel elevated) can be told from a few argmax
flips (a handful of channels)."""
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import mpi_cuda_cnn_amd as mcc  # noqa: E402
from mpi_cuda_cnn_amd.models.torch_reference import TorchReference, images_to_nchw  # noqa: E402
from tests.test_gpu_engine import _BIG_SPECS, _per_channel_err  # noqa: E402


def run(spec, dtype, B, seed, dev):
    C, H, W = spec.input_shape()
    imgs, labels = mcc.synth_dataset(B, C, H, W, spec.num_classes(), seed=seed)
    params = mcc.init_params(spec, seed=1).astype(np.float32)
    net = mcc.GpuNet(spec, dtype, B)
    net.set_params(params)
    d_img = torch.from_numpy(imgs).to(dev)
    d_lab = torch.from_numpy(labels).to(dev)
    s = torch.cuda.current_stream().cuda_stream
    net.forward(d_img.data_ptr(), 0, B, s)
    net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
    net.backward_all(s)
    torch.cuda.synchronize()
    grads = net.get_grads()
    plan = net.plan()
    mimic = dtype == "bf16"
    ref = TorchReference(spec, dtype=torch.float64, mimic_bf16=mimic)
    ref.load_flat(torch.from_numpy(params.astype(np.float64)))
    x = images_to_nchw(imgs, torch.float64)
    if mimic and "fwd:s1" not in plan:
        x = x.to(torch.bfloat16).to(torch.float64)
    logits = ref(x)
    F.cross_entropy(logits, torch.from_numpy(labels.astype(np.int64))).backward()
    rg = ref.flat_grads().numpy()
    print(f"== {dtype}: logits rel err {np.linalg.norm(net.get_logits(B) - logits.detach().numpy()) / np.linalg.norm(logits.detach().numpy()):.2e}")
    for L in spec.layers():
        if L["nweights"] == 0:
            continue
        for off, n, what in ((L["w_off"], L["nweights"], "W"), (L["b_off"], L["nbiases"], "b")):
            g = grads[off : off + n].reshape(L["C"], -1).astype(np.float64)
            r = rg[off : off + n].reshape(L["C"], -1)
            rn = np.linalg.norm(r, axis=1)
            floor = (0.3 if what == "b" else 1e-2) * np.linalg.norm(r) / np.sqrt(L["C"])
            e = np.linalg.norm(g - r, axis=1) / np.maximum(rn, max(floor, 1e-30))
            q = np.quantile(e, [0.5, 0.99])
            print(f"  {L['kind']} C={L['C']} {what}: max {e.max():.2e} (ch {int(e.argmax())}) p99 {q[1]:.2e} "
                  f"median {q[0]:.2e}  #>5e-2: {int((e > 5e-2).sum())}")


if __name__ == "__main__":
    name = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    spec = mcc.parse_model_spec(_BIG_SPECS[name], name) if name in _BIG_SPECS else mcc.make_model(name)
    dev = torch.device("cuda", 0)
    for dt in ("fp32", "bf16"):
        run(spec, dt, B, seed, dev)
