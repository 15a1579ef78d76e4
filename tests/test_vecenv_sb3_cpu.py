"""CPU: SmartNanogridVecEnv's class hierarchy with and without stable-baselines3.

SB3's BaseAlgorithm._wrap_env accepts a batched env only through `isinstance(env, VecEnv)` and wraps
anything else in DummyVecEnv as one env (the reference attaches its env that way,
solvers/RL/ppo_train.py:89-92).  With SB3 importable the class must derive from SB3's VecEnv and leave
no abstract method unimplemented; without it the base is `object` (this image).  SB3 2.x's seed() /
set_options() semantics (kept for the next reset) are checked here on a handle-less instance; the GPU
side runs in tests/test_gpu_vecenv_api.py.  SB3 itself is absent, so this is against a stand-in of its
abstract VecEnv (tests/sb3_stub.py): the SB3 runtime is parity-unpinned.
"""
import importlib.util

import pytest

from sb3_stub import VecEnv, load_vec_env_with_sb3


def test_without_sb3_the_base_is_object():
    assert importlib.util.find_spec("stable_baselines3") is None
    from smart_nanogrid_gym import vec_env
    assert vec_env._VecEnvBase is object
    assert vec_env.SmartNanogridVecEnv.__bases__ == (object,)


def test_with_sb3_the_class_is_an_sb3_vecenv():
    mod = load_vec_env_with_sb3()
    cls = mod.SmartNanogridVecEnv
    assert mod._VecEnvBase is VecEnv
    assert issubclass(cls, VecEnv)
    assert not getattr(cls, "__abstractmethods__", frozenset())   # every abstract method implemented
    # the package's own module is untouched
    from smart_nanogrid_gym import SmartNanogridVecEnv
    assert not issubclass(SmartNanogridVecEnv, VecEnv)


def _bare(cls, n):
    v = cls.__new__(cls)
    v.num_envs = n
    v.env_offset = 0
    v.rng_mode = 0   # _native.RNG_REFERENCE
    v._seeds = [None] * n
    v._options = [{} for _ in range(n)]
    return v


@pytest.mark.parametrize("with_sb3", [False, True])
def test_seed_and_options_wait_for_the_next_reset(with_sb3):
    if with_sb3:
        cls = load_vec_env_with_sb3().SmartNanogridVecEnv
    else:
        from smart_nanogrid_gym import SmartNanogridVecEnv as cls
    v = _bare(cls, 4)
    assert v.seed(11) == [11, 12, 13, 14]
    assert v._seeds == [11, 12, 13, 14]
    s = v.seed()
    assert s == [s[0] + i for i in range(4)] and 0 <= s[0] and s[-1] < 2 ** 32
    # reference-RNG env i is np.random.seed(seed + env_offset + i), numpy's range is [0, 2^32)
    assert v.seed(2 ** 32 - 4)[-1] == 2 ** 32 - 1
    for bad in (2 ** 32 - 3, -1):
        with pytest.raises(ValueError, match="2\\*\\*32"):
            v.seed(bad)
    v.env_offset = 1000
    with pytest.raises(ValueError):
        v.seed(2 ** 32 - 1000)
    for _ in range(200):   # a fresh seed keeps every env's seed in range
        assert v.seed()[-1] + v.env_offset < 2 ** 32
    v.env_offset = 0
    v.set_options({"generate_new_initial_values": False})
    assert v._options == [{"generate_new_initial_values": False}] * 4
    v.set_options()
    assert v._options == [{}] * 4
    with pytest.raises(ValueError):
        v.set_options([{}] * 3)
    # options that differ per env or that reset() does not take are refused at the reset, before any GPU work
    v.set_options([{"generate_new_initial_values": i % 2 == 0} for i in range(4)])
    with pytest.raises(ValueError, match="resets alike"):
        v.reset()
    v.set_options({"no_such_option": 1})
    with pytest.raises(ValueError, match="unknown reset options"):
        v.reset()
