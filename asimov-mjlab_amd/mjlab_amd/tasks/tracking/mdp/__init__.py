from mjlab_amd.envs.mdp import *  # noqa: F401,F403
from mjlab_amd.tasks.tracking.mdp.commands import *  # noqa: F401,F403
from mjlab_amd.tasks.tracking.mdp.observations import *  # noqa: F401,F403
from mjlab_amd.tasks.tracking.mdp.rewards import *  # noqa: F401,F403
from mjlab_amd.tasks.tracking.mdp.terminations import *  # noqa: F401,F403
