from mjlab_amd.tasks import register
from mjlab_amd.tasks.tracking.config.g1 import (
  unitree_g1_flat_tracking_env_cfg,
  unitree_g1_flat_tracking_no_state_estimation_env_cfg,
)

register("Mjlab-Tracking-Flat-Unitree-G1", unitree_g1_flat_tracking_env_cfg)
register("Mjlab-Tracking-Flat-Unitree-G1-No-State-Estimation", unitree_g1_flat_tracking_no_state_estimation_env_cfg)
