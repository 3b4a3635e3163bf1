"""Sentinels shared by the host API and the device tables (reference `utils/constants.py:1-4`).

The same values are compiled into the kernels (`csrc/rt_device.h`: RT_FARAWAY, RT_SKYBOX_DISTANCE).
"""
UPWARDS = 1
UPDOWN = -1
FARAWAY = 1.0e39
SKYBOX_DISTANCE = 1.0e6
