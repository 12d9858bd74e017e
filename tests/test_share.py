"""ShareData host side: stop flags and the tracked
trajectory across processes, pickling by name, layout checks.  The device
snapshots themselves are covered by tests/test_gpu_share.py.

Reference behaviour followed: src/share.py:27-166 (properties, push_pose /
tracking_trajectory), voxslam.py:28-33 (one shared object handed to both
processes), tracking.py:105, :159 (stop_mapping, push_pose of the
translation)."""
import multiprocessing as mp
import os
import pickle

import numpy as np
import pytest
import torch

from psvo.share import ShareData


def _child(share, q):
    # attached by name through pickling, like the reference's manager proxy
    q.put((share.stop_mapping, share.stop_tracking, [p.tolist() for p in share.tracking_trajectory]))
    share.push_pose(np.array([7.0, 8.0, 9.0]))
    share.stop_mapping = True
    share.close()


def test_flags_and_trajectory_cross_process():
    s = ShareData()
    try:
        s.stop_tracking = True
        s.push_pose([1.0, 2.0, 3.0])
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=_child, args=(s, q))
        p.start()
        seen = q.get(timeout=120)
        p.join(timeout=120)
        assert p.exitcode == 0
        assert seen == (False, True, [[1.0, 2.0, 3.0]])
        assert s.stop_mapping is True
        traj = s.tracking_trajectory
        assert [t.tolist() for t in traj] == [[1.0, 2.0, 3.0], [7.0, 8.0, 9.0]]
    finally:
        s.close()
    assert not any(s.name[1:] in f for f in os.listdir("/dev/shm"))


def test_pickle_attaches_same_block():
    s = ShareData()
    try:
        t = pickle.loads(pickle.dumps(s))
        assert t.name == s.name
        t.push_pose([0.5, -1.0, 2.0, 3.0, 4.0, 5.0, 6.0])   # up to 7 numbers (translation + quaternion)
        assert s.tracking_trajectory[0].tolist() == [0.5, -1.0, 2.0, 3.0, 4.0, 5.0, 6.0]
        with pytest.raises(RuntimeError):
            t.push_pose(np.zeros(8))
        t.close()
        assert s.version("states") == 0
    finally:
        s.close()


def test_rejects_unshareable_values():
    s = ShareData()
    try:
        with pytest.raises(TypeError):
            s.states = {"voxel_center_xyz": [1, 2, 3]}
        with pytest.raises(TypeError):
            s.octree = object()
    finally:
        s.close()


def test_attach_missing_segment_raises():
    with pytest.raises(RuntimeError):
        ShareData("/psvo-share-does-not-exist", _attach=True)
