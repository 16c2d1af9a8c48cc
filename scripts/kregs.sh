#!/bin/bash
# VGPR / AGPR / VGPR-spill / LDS / occupancy per kernel of a libhgk source (compiler remarks)
# usage: scripts/kregs.sh hgk_conv [pattern]
src=${1:-hgk_conv}; pat=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Iinclude --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage -Wno-inline-asm \
  $EXTRA progressive_process_for_human_pose_estimation_amd/csrc/$src.hip -o /dev/null 2>&1 | \
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass.*//' | \
  awk '/^Function Name:/{n=$3} /^VGPRs:/{v=$2} /^AGPRs:/{ag=$2} /^Occupancy/{oc=$NF} /^VGPRs Spill:/{sp=$NF} /^LDS Size/{print "vgpr="v, "agpr="ag, "spill="sp, "occ="oc, "lds="$NF, n}' | \
  c++filt | grep -- "$pat"
