#!/bin/bash
# features of the in-tree library against tools/probes/_old/libcasr_hip.so (a build of the previous
# commit), bit for bit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 200 python tools/probes/feat_bitwise.py tools/probes/_old/libcasr_hip.so /tmp/casr_feat_old.npz &&
timeout -k 10 200 python tools/probes/feat_bitwise.py chinese-asr_amd/casr/libcasr_hip.so /tmp/casr_feat_new.npz &&
python -c "
import numpy as np
a=np.load('/tmp/casr_feat_old.npz'); b=np.load('/tmp/casr_feat_new.npz')
for k in a.files: print(k, a[k].shape, 'bitwise equal' if np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)) else 'DIFFER')"
