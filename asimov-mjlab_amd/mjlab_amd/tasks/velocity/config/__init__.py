from mjlab_amd.tasks import register
from mjlab_amd.tasks.velocity.config.g1 import unitree_g1_flat_env_cfg
from mjlab_amd.tasks.velocity.config.go1 import unitree_go1_flat_env_cfg

register("Mjlab-Velocity-Flat-Unitree-G1", unitree_g1_flat_env_cfg)
register("Mjlab-Velocity-Flat-Unitree-Go1", unitree_go1_flat_env_cfg)
