"""Per-bucket SGD (GpuNet.sgd_range, BucketedAllReduce.backward_update) is
bit-identical to the whole-buffer update.

At world > 1 a data-parallel step updates each gradient bucket's parameters
as soon as that bucket's all-reduce has landed, so the LeNet-5 FC update
(96 % of the bytes) runs while the conv block's small collective -- issued
after the fused conv-block backward -- is still in flight (the reference
joined every MPI_Allreduce before its update, cnnmpi.c:487-499).  The SGD is
elementwise, so splitting it by range must not change a single bit: checked
here in one process (no process group: the per-bucket path still runs),
across the engine's three SGD code paths -- the fused SGD + packed-copy
refresh with elementwise stages, with a tiled (transposing) conv stage
(CIFAR-3conv conv3, 73,728 weights >= the tile threshold), and the
gather-table path (MCC_AB=no_fused_pack) -- with momentum and weight decay.
"""

import numpy as np
import pytest
import torch

import mpi_cuda_cnn_amd as mcc

STEPS = 3


def _run(model, dtype, B, split, monkeypatch, ab=None):
    from mpi_cuda_cnn_amd.trainer import GpuTrainer

    if ab:
        monkeypatch.setenv("MCC_AB", ab)
    else:
        monkeypatch.delenv("MCC_AB", raising=False)
    spec = mcc.make_model(model)
    C, H, W = spec.input_shape()
    imgs, labels = mcc.synth_dataset(STEPS * B, C, H, W, spec.num_classes(), seed=11)
    dev = torch.device("cuda", 0)
    d_img, d_lab = torch.from_numpy(imgs).to(dev), torch.from_numpy(labels).to(dev)
    tr = GpuTrainer(spec, dtype=dtype, batch=B, device=0, lr=0.05, momentum=0.9, weight_decay=1e-4,
                    params=mcc.init_params(spec, seed=3), bucket_bytes=4096, split_sgd=split)
    nb = len(tr.sync.buckets)
    for s in range(STEPS):
        idx = torch.arange(s * B, (s + 1) * B, device=dev, dtype=torch.int32)
        tr.step(d_img, d_lab, idx)
    torch.cuda.synchronize()
    # the packed compute copies too: one more forward's logits
    s = torch.cuda.current_stream().cuda_stream
    idx = torch.arange(0, B, device=dev, dtype=torch.int32)
    tr.net.forward(d_img.data_ptr(), idx.data_ptr(), B, s)
    torch.cuda.synchronize()
    return tr.state_dict(), tr.net.get_logits(B), nb


@pytest.mark.gpu
@pytest.mark.parametrize("model,dtype,B,ab", [
    ("lenet5", "bf16", 256, None),
    ("lenet5", "fp32", 256, None),
    ("ref", "bf16", 256, None),
    ("cifar3", "bf16", 128, None),
    ("lenet5", "bf16", 256, "no_fused_pack"),
])
def test_split_sgd_bit_equal(model, dtype, B, ab, monkeypatch):
    ps, ls, nb = _run(model, dtype, B, True, monkeypatch, ab)
    pj, lj, _ = _run(model, dtype, B, False, monkeypatch, ab)
    assert nb > 1, "needs several buckets"
    np.testing.assert_array_equal(ps, pj)
    np.testing.assert_array_equal(ls, lj)


@pytest.mark.gpu
def test_sgd_range_rejects_partial_stage():
    spec = mcc.make_model("lenet5")
    net = mcc.GpuNet(spec, "bf16", 64)
    off, cnt = net.stage_param_range(2)
    with pytest.raises(Exception):
        net.sgd_range(0.1, 0.0, 0.0, off + 1, cnt - 1, 0)
