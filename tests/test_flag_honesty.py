"""Flags do what they say: ``--dtype fp32`` never runs the bf16 kernels,
``--test`` without a checkpoint fails unless ``--allow_random_init``."""
import pytest
import torch

from microbeast_amd.cli import main
from microbeast_amd.config import parse_flags
from microbeast_amd.models.factory import make_model


@pytest.mark.parametrize("arch", ["impala_flat", "gridnet"])
def test_fp32_model_has_no_hip_path(arch):
    f = parse_flags(["--dtype", "fp32", "--arch", arch, "--env_size", "8"], interactive=False)
    m = make_model(f)
    assert m.compute_dtype == torch.float32 and m.hip_kernels is False
    b = make_model(parse_flags(["--arch", arch, "--env_size", "8"], interactive=False))
    assert b.compute_dtype == torch.bfloat16 and b.hip_kernels is True


def test_unknown_dtype_raises():
    with pytest.raises(ValueError):
        make_model(parse_flags(["--dtype", "fp16"], interactive=False))


def test_gpu_runtime_refuses_fp32(tmp_path):
    from microbeast_amd.train import train

    f = parse_flags(["--runtime", "gpu", "--dtype", "fp32", "--savedir", str(tmp_path),
                     "--exp_name", "x"], interactive=False)
    with pytest.raises(ValueError, match="fp32"):
        train(f)


def test_test_mode_without_checkpoint_fails(tmp_path):
    base = ["--test", "--exp_name", "nock", "--savedir", str(tmp_path), "--device", "cpu",
            "--env_size", "4", "--n_envs", "2", "--eval_episodes", "1",
            "--max_episode_steps", "20"]
    assert main(base) != 0
    assert not (tmp_path / "nock_eval.csv").exists()
    assert main(base + ["--allow_random_init"]) == 0
    assert (tmp_path / "nock_eval.csv").exists()


def test_gpu_runtime_refuses_real_env(tmp_path):
    """the GPU engine steps the native stand-in only, so ``--env microrts``
    on it must fail loudly instead of silently training on the stand-in."""
    from microbeast_amd.train import train

    f = parse_flags(["--runtime", "gpu", "--env", "microrts", "--savedir", str(tmp_path),
                     "--exp_name", "x"], interactive=False)
    with pytest.raises(ValueError, match="--env microrts is not available on the gpu runtime"):
        train(f)


def test_auto_runtime_routes_real_env_to_mono():
    """``--runtime auto --env microrts`` picks the CPU actor runtime, whose actor processes
    build the gym-microrts adapter (runtime/mono.py passes ``env=flags.env`` to create_env);
    the adapter refuses loudly when gym-microrts is absent."""
    from microbeast_amd.envs.synthetic import create_env
    from microbeast_amd.train import resolve_runtime

    real = parse_flags(["--env", "microrts"], interactive=False)
    assert resolve_runtime(real, want_cuda=True) == "mono"
    assert resolve_runtime(real, want_cuda=False) == "mono"
    stand_in = parse_flags([], interactive=False)
    assert resolve_runtime(stand_in, want_cuda=True) == "gpu"
    from microbeast_amd.envs.microrts import gym_microrts_available

    if not gym_microrts_available():
        with pytest.raises(RuntimeError, match="gym-microrts"):
            create_env(4, 2, 20, env="microrts")


def test_unknown_env_raises(tmp_path):
    from microbeast_amd.train import train

    f = parse_flags(["--env", "atari", "--savedir", str(tmp_path), "--exp_name", "x"],
                    interactive=False)
    with pytest.raises(ValueError, match="--env"):
        train(f)
