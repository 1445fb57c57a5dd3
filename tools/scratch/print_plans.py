"""Print the engine's per-stage kernel plan for a few model/dtype pairs (GPU box)."""
import sys
import mpi_cuda_cnn_amd as m

pairs = [a.split(":") for a in sys.argv[1:]] or [("lenet5", "bf16"), ("lenet5", "fp32"), ("cifar3", "bf16"),
                                                 ("vgg11", "bf16")]
for name, dt in pairs:
    net = m.GpuNet(m.make_model(name), dt, 64)
    print(name, dt)
    print(net.plan())
