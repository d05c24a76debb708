"""Host fast paths of the dispatch layer: the raw current-stream handle used for every kernel
launch equals torch's current stream (default, side and high-priority streams), and the cached
config flags follow config.set_property."""
import pytest
import torch


def test_cached_flags_follow_set_property():
    from bigdl.nn import abstractnn
    from bigdl.ops import native
    from bigdl.utils import config
    config.set_property("bigdl.native.enable", False)
    assert not native.has("conv2d_forward")
    config.clear_property("bigdl.native.enable")
    assert native._ENABLED[0] == bool(config.get_property("bigdl.native.enable"))
    config.set_property("bigdl.profile.sync", True)
    assert abstractnn._PROFILE_SYNC[0]
    config.set_property("bigdl.profile.sync", False)
    assert not abstractnn._PROFILE_SYNC[0]


@pytest.mark.gpu
def test_raw_stream_pointer_matches_torch():
    from bigdl.ops.native import stream_ptr
    assert stream_ptr() == torch.cuda.current_stream().cuda_stream
    for prio in (0, -1):
        s = torch.cuda.Stream(priority=prio)
        with torch.cuda.stream(s):
            assert stream_ptr() == s.cuda_stream == torch.cuda.current_stream().cuda_stream
    assert stream_ptr() == torch.cuda.current_stream().cuda_stream
