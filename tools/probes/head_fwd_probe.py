"""fused-forward xent head vs the separate last-FC forward (MCC_AB=no_head_fwd): logits of one step."""
import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
import mpi_cuda_cnn_amd as mcc
model, dtype, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
spec = mcc.make_model(model)
C, H, W = spec.input_shape()
imgs, labels = mcc.synth_dataset(B, C, H, W, spec.num_classes(), seed=3)
params = mcc.init_params(spec, seed=1).astype(np.float32)
net = mcc.GpuNet(spec, dtype, B)
print(net.plan())
net.set_params(params)
d_img = torch.from_numpy(imgs).cuda(); d_lab = torch.from_numpy(labels).cuda()
s = torch.cuda.current_stream().cuda_stream
net.zero_stats(s); net.forward(d_img.data_ptr(), 0, B, s); net.loss(d_lab.data_ptr(), 0, 1.0 / B, True, s)
torch.cuda.synchronize()
lg = net.get_logits(B)
print(os.environ.get("MCC_AB"), "nan", int(np.isnan(lg).sum()), "rows with nan", np.where(np.isnan(lg).any(1))[0][:10], lg[:2])
np.save(f"gpurun_out/headprobe_{os.environ.get('MCC_AB','on')}.npy", lg)
