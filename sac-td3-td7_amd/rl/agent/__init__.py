from rl.agent.abc import Agent  # noqa: F401
from rl.agent.sac import SAC  # noqa: F401
from rl.agent.td3 import TD3  # noqa: F401
from rl.agent.td7 import TD7  # noqa: F401
