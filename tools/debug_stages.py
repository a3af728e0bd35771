"""Compare per-stage engine buffers with the reference's forward-hook intermediates."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'mswe-gnn_amd'), os.path.join(ROOT, 'oracle')]
import numpy as np, torch
from conftest import build_msgnn, golden, weights, rel_err
from mswegnn.mesh import make_multiscale_mesh, wet_state, mesh_config
from mswegnn.engine import plan_for
ck, K, F = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 1 else ("K4_F32", 4, 32)
fx = golden(f"fx_tiny_{ck}_step")
dev = torch.device('cuda:0')
g = wet_state(make_multiscale_mesh(**mesh_config("tiny"), T=48), seed=1).to(dev)
m = build_msgnn(4, F, K, state=weights(ck)).to(dev); m.engine = 'hip'
with torch.no_grad(): y = m(g)
plan = plan_for(m, g)
np_ = g.node_ptr.cpu().tolist()
xd = plan.debug_buffer('x_down', F).cpu(); xu = plan.debug_buffer('x_up', F).cpu()
for i in range(3):
    a, b = np_[i], np_[i+1]
    ref = fx[f'mid__gnn_processor_{i}'][a:b]
    print(f'proc{i} scale{i}: rel {rel_err(xd[a:b], ref):.3e}  max|ref| {np.abs(ref).max():.3f}')
for i in range(4):
    s = 3 - i; a, b = np_[s], np_[s+1]
    ref = fx[f'mid__gnn_processor_{3+i}'][a:b]
    print(f'proc{3+i} scale{s}: rel {rel_err(xu[a:b], ref):.3e}  max|ref| {np.abs(ref).max():.3f}')
print('y rel', rel_err(y.cpu(), fx['y']))
