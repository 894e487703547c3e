from rl.utils.envs import get_action_bias_scale, get_state_action_dims, register_env  # noqa: F401
