"""The Ceres cost-functor boundary from C++: tests/cpp/test_factors.cpp builds
residual blocks through the reference functors' Create() (include/lislam_factors.h, signatures of
lidarFeaturePointsFunction.hpp:21-293), evaluates them on the GPU via CostFunction::Evaluate and
one batched lislam::EvaluateBlocks launch, and compares residuals and raw-parameter Jacobians with
the oracle's Ceres-Jet autodiff (residual 1e-12, Jacobian 1e-9 relative); then a 2,304-block
problem (laserOdometry's size) evaluated block by block as Ceres does, one launch per parameter
point (lidarFeaturePointsFunction.hpp:49-54,183-190,282-288 batched).  The binary is built by
__graft_entry__.build() (g++, no ROS, linked against liblislam.so)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_factors")


def test_cpp_consumer_is_built():
    assert os.path.exists(BIN), "run __graft_entry__.build() first"


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_cpp_functor_create_evaluate_on_gpu():
    out = subprocess.run([BIN], capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "factors ok: 200 blocks" in out.stdout
    # Ceres' per-block Evaluate() over a 2,304-block problem: one launch per parameter point
    assert "batched: 2304 blocks, 5 parameter points, 1 launch each" in out.stdout
