"""How long does the reference loss head (decoder + nll_loss + reg_loss, fwd+bwd) take
in plain torch on the state49 batch?  (sizing the fused-epilogue row of SURVEY 8f)"""
import sys, time
sys.path.insert(0, "/root/repo")
import importlib, torch
importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
import lib.models as models, lib.train_functions as tf
dev = "cuda"
T, S, B, R, L = 9, 64, 320, 49, 8
lat = torch.randn(T, S * B, R, L, device=dev).requires_grad_(True)
dec = models.Decoder(R, L, 1).to(dev)
y = torch.rand(B, T, R, device=dev)
def step():
    yp = dec(lat[..., :3]).reshape((-1, S, B, R)).permute(2, 1, 0, 3)
    loss = tf.nll_loss(yp, y) + 0.1 * tf.latent_init_loss(lat[..., :3])
    loss.backward()
for _ in range(3): step()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(20): step()
torch.cuda.synchronize(); print("loss head fwd+bwd ms", (time.perf_counter() - t0) / 20 * 1e3)
from ude_amd import loss_head
ode = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd").FaFp(
    R, latent_dim=L, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(dev)
lin = dec.decoder[-1]
def fstep():
    nll, reg = loss_head.fused_loss_head(ode, lat, lin, y, S, B)
    (nll + 0.1 * reg).backward()
for _ in range(3): fstep()
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(20): fstep()
torch.cuda.synchronize(); print("fused loss head fwd+bwd ms", (time.perf_counter() - t0) / 20 * 1e3)
