#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-bnstamps}; mkdir -p $O
export PYTHONPATH=$PWD/multi-camera_3d_pose_estimation_amd
MVPOSE_LIB=multi-camera_3d_pose_estimation_amd/mvpose/libbn_stamps.so timeout -k 10 120 python -u tools/bneck_stamps.py > $O/stamps.txt 2>&1; rc=$?; cat $O/stamps.txt; exit $rc
