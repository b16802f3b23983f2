"""Probe: can two RCCL ranks share one GPU (for testing the partitioned path on a 1-GPU box)?"""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd")); sys.path.insert(0, ROOT)
import torch.distributed as dist
rank = int(os.environ["RANK"]); world = int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
from tvfem import box_mesh, _native as N
from tvfem.problem import ThermoViscoProblem
mp = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0, "htc": 280.1,
      "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0, "Rg": 8.314, "alpha_solid": 9.1e-6, "alpha_liquid": 25.1e-6}
cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
mesh = box_mesh([2.0, 4.0, 1.0], [8, 16, 4])
prob = ThermoViscoProblem(mesh, (0, 1), 0.1, cfg, mp, device=0, n_parts=world, part=rank, part_axis=1, verbose=False, write_output=False)
lib, ctx = prob._lib, prob._ctx
buf = C.create_string_buffer(lib.tv_comm_unique_id_size())
if rank == 0:
    N.check(lib.tv_comm_get_unique_id(buf))
obj = [buf.raw if rank == 0 else None]
dist.broadcast_object_list(obj, src=0)
rc = lib.tv_comm_init(ctx, C.c_char_p(obj[0]), world, rank)
print(rank, "comm_init rc", rc, lib.tv_last_error(ctx), flush=True)
if rc == 0:
    prob.setup()
    for _ in range(3):
        prob.solve_timestep()
    T = prob.functions_current["T"].x.array
    print(rank, "T", T.min(), T.max(), prob.last_newton_iterations, prob.last_krylov_iterations, flush=True)
prob.close()
