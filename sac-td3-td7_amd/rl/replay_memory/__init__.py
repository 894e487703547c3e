from rl.replay_memory.base import BaseReplayMemory, DeviceBatch  # noqa: F401
from rl.replay_memory.lap import LAPReplayMemory  # noqa: F401
from rl.replay_memory.simple import SimpleReplayMemory  # noqa: F401
