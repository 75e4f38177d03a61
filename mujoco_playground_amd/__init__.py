"""mujoco_playground_amd: MI355X-native batched physics step for the ackermann_robot_v2 env.

Hot path: libackphys.so (HIP, gfx950) behind the C-ABI in include/ackphys.h; host side in
Python (sim.BatchedAckermannSim, rl.AckermannVecEnv, rl.AckermannRobotEnv).
"""
__version__ = "0.1.0"
