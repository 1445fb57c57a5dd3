"""Print the engine's per-stage kernel plan for a few model/dtype pairs (GPU box)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import mpi_cuda_cnn_amd as m  # noqa: E402

pairs = [a.split(":") for a in sys.argv[1:]] or [("lenet5", "bf16"), ("lenet5", "fp32"), ("cifar3", "bf16"),
                                                 ("vgg11", "bf16")]
for name, dt in pairs:
    net = m.GpuNet(m.make_model(name), dt, 64)
    print(name, dt)
    print(net.plan())
