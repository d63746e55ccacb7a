from mjlab_amd.envs.mdp.actions import JointPositionAction, JointPositionActionCfg  # noqa: F401
from mjlab_amd.envs.mdp.events import *  # noqa: F401,F403
from mjlab_amd.envs.mdp.observations import *  # noqa: F401,F403
from mjlab_amd.envs.mdp.rewards import *  # noqa: F401,F403
from mjlab_amd.envs.mdp.terminations import *  # noqa: F401,F403
