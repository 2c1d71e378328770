#!/bin/bash
# Where the GPU box exposes board power / clocks in sysfs (read only).
for d in /sys/bus/pci/devices/*/hwmon/hwmon*; do
  [ -e "$d/name" ] || continue
  echo "== $d ($(cat $d/name 2>/dev/null))"
  for f in $d/power1_* $d/freq1_* $d/in0_* $d/temp1_input; do
    [ -e "$f" ] && echo "$f: $(cat $f 2>/dev/null)"
  done
done
ls /sys/class/drm/ 2>/dev/null | head -20
