"""Scripted goal-seeking controller on the batched env (GPU): a = [1, clip(2*goal_angle)].
Shows how far the robot gets per episode length (timestep 2 ms, one mj_step per env.step), i.e.
whether goals 2-8 m away are reachable within the reference's 1000-step episodes (they are not).
    python tools/probes/drive_check.py
"""
import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mujoco_playground_amd.rl import make_ackermann_env
dev = torch.device('cuda:0')
env = make_ackermann_env(env_type="vec", num_envs=1024, device=dev, seed=5, max_episode_steps=3000, collision_threshold=-2)
sim = env.sim
obs = env.reset()
p0 = sim.state[0:3].clone()
done = torch.zeros(1024, dtype=torch.bool, device=dev)
for t in range(3000):
    o = sim.obs_soa
    ang = o[78]; dist = o[77]
    a = torch.stack([torch.full_like(ang, 1.0), torch.clamp(2.0 * ang, -1, 1)], dim=1)
    sim.step(a.contiguous(), autoreset=False, want_info=False, want_terminal=False, track_episodes=False)
    done |= sim.term.bool()
    if t in (99, 499, 999, 2999):
        torch.cuda.synchronize()
        print(t+1, 'success frac', float(done.float().mean()), 'mean dist', float(sim.obs_soa[77].mean()), 'moved', float((sim.state[0:2]-p0[0:2]).norm(dim=0).mean()), 'z', float(sim.state[2].mean()))
