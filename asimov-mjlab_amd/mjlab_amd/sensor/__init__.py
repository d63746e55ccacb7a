from mjlab_amd.sensor.builtin_sensor import BuiltinSensor
from mjlab_amd.sensor.contact_sensor import (
  ContactData,
  ContactMatch,
  ContactSensor,
  ContactSensorCfg,
  SensorCfg,
)

__all__ = ["BuiltinSensor", "ContactData", "ContactMatch", "ContactSensor", "ContactSensorCfg", "SensorCfg"]
