from gym_macm.envs.mvmnt import Flock  # noqa: F401
from gym_macm.envs.combat import TDM, ControlledTDM  # noqa: F401
