"""Checkpoint / resume of a batch (the reference never checkpoints env
state; the build's snapshot makes it trivial).  A batch saved mid-run and restored into a new
env continues bit-identically: every draw is keyed by the seed, the global env id and the
per-env counter the snapshot carries."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env_id", ["DroneHoverBulletFreeEnvWithGust-v0", "DroneHoverBulletEnvWithRandomAdversary-v0"])
def test_resume_from_checkpoint_is_bit_identical(gpu, tmp_path, env_id):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 3000
    a_env = BatchedCrazyflieEnv(env_id, n, seed=8, env_id_offset=512, want_final_obs=True)
    a_env.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(2)
    acts = [(torch.rand(n, 4, device="cuda", generator=gen) * 2 - 1).contiguous() for _ in range(40)]
    for t in range(20):
        a_env.step(acts[t])
    path = str(tmp_path / "batch.safetensors")
    a_env.save_checkpoint(path)
    b_env = BatchedCrazyflieEnv.from_checkpoint(path)
    assert b_env.num_envs == n and b_env.want_final_obs
    np.testing.assert_array_equal(b_env.obs.cpu().numpy(), a_env.obs.cpu().numpy())
    dones = 0
    for t in range(20, 40):
        oa, ra, da, ia = a_env.step(acts[t])
        ob, rb, db, ib = b_env.step(acts[t])
        np.testing.assert_array_equal(ob.cpu().numpy(), oa.cpu().numpy())
        np.testing.assert_array_equal(rb.cpu().numpy(), ra.cpu().numpy())
        np.testing.assert_array_equal(db.cpu().numpy(), da.cpu().numpy())
        m = da.cpu().numpy().astype(bool)              # final_obs rows are written for finished envs only
        np.testing.assert_array_equal(ib["final_obs"].cpu().numpy()[m], ia["final_obs"].cpu().numpy()[m])
        dones += int(da.sum())
    assert dones > 0                                   # resets (fresh draws) happened after the resume
    for x, y in zip(a_env.get_state(), b_env.get_state()):
        np.testing.assert_array_equal(x.cpu().numpy(), y.cpu().numpy())
    # a differently configured env refuses the checkpoint
    other = BatchedCrazyflieEnv(env_id, n, seed=9, env_id_offset=512)
    with pytest.raises(ValueError):
        other.load_checkpoint(path)
    for e in (a_env, b_env, other):
        e.close()


@pytest.mark.parametrize("path_kind", ["rollout", "step_into"])
def test_checkpoint_after_rollout_or_step_into_resumes(gpu, tmp_path, path_kind):
    """rollout() and step_into() write the observations into caller buffers; the checkpoint then
    saves those (the latest step's), not the env's own obs buffer, and a resumed batch continues
    bit-identically (self.obs used to be stale there)."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id, n = "DroneHoverBulletFreeEnvWithGust-v0", 2048
    a_env = BatchedCrazyflieEnv(env_id, n, seed=4)
    a_env.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    acts = (torch.rand(16, n, 4, device="cuda", generator=gen) * 2 - 1).contiguous()
    if path_kind == "rollout":
        obs, _, _, _ = a_env.rollout(acts[:8])
        latest = obs[7].clone()
    else:
        ob = torch.empty(n, a_env.obs_dim, device="cuda")
        rw = torch.empty(n, device="cuda")
        dn = torch.empty(n, dtype=torch.uint8, device="cuda")
        for t in range(8):
            a_env.step_into(acts[t], ob, rw, dn)
        latest = ob.clone()
    path = str(tmp_path / "b.safetensors")
    a_env.save_checkpoint(path)
    b_env = BatchedCrazyflieEnv.from_checkpoint(path)
    np.testing.assert_array_equal(b_env.obs.cpu().numpy(), latest.cpu().numpy())
    for t in range(8, 16):
        oa, ra, da, _ = a_env.step(acts[t])
        ob2, rb, db, _ = b_env.step(acts[t])
        np.testing.assert_array_equal(ob2.cpu().numpy(), oa.cpu().numpy())
        np.testing.assert_array_equal(rb.cpu().numpy(), ra.cpu().numpy())
    # observations sent to a raw pointer: the checkpoint needs them explicitly
    raw = torch.empty(n, a_env.obs_dim, device="cuda")
    a_env.step_raw(acts[0].data_ptr(), obs_ptr=raw.data_ptr())
    with pytest.raises(ValueError, match="obs="):
        a_env.save_checkpoint(path)
    a_env.save_checkpoint(path, obs=raw)
    for e in (a_env, b_env):
        e.close()
