"""MI355X engine-backed mirror of the reference's ``rl`` package hot path.

Agents (``rl.agent.TD7/TD3/SAC``), device replay memories
(``rl.replay_memory.LAPReplayMemory/SimpleReplayMemory``) and
``rl.runner.run_train_ops`` keep the reference's interface; every gradient step
runs in ``lib/librle.so`` (HIP, gfx950) through the C ABI in include/rle.h.
"""
