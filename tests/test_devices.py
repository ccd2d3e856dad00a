"""GPU counting without HIP (ddpx.utils.devices): environment and KFD-topology rules."""
import os

from ddpx.utils import devices


def _node(root, i, simd, minor):
    d = root / "nodes" / str(i)
    d.mkdir(parents=True)
    (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {simd}\ndrm_render_minor {minor}\n")


def test_kfd_count_keeps_granted_render_nodes(tmp_path):
    dri = tmp_path / "dri"
    dri.mkdir()
    _node(tmp_path, 0, 0, 0)  # CPU node
    for i, minor in enumerate([128, 136, 144], start=1):
        _node(tmp_path, i, 1024, minor)
    (dri / "renderD128").write_text("")
    (dri / "renderD144").write_text("")
    assert devices.kfd_gpu_count(str(tmp_path / "nodes"), str(dri)) == 2
    assert devices.kfd_gpu_count(str(tmp_path / "missing"), str(dri)) is None


def test_env_count_rules():
    assert devices._env_count({}) is None
    assert devices._env_count({"HIP_VISIBLE_DEVICES": "0,3"}) == 2
    assert devices._env_count({"ROCR_VISIBLE_DEVICES": ""}) == 0
    assert devices._env_count({"HIP_VISIBLE_DEVICES": "0,1,2", "CUDA_VISIBLE_DEVICES": "1"}) == 1


def test_visible_count_prefers_env_without_hip(monkeypatch):
    monkeypatch.setattr(devices, "kfd_gpu_count", lambda *a, **k: 8)
    assert devices.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert devices.visible_gpu_count({}) == 8
    import torch
    assert not torch.cuda.is_initialized()
    assert os.environ is not None
