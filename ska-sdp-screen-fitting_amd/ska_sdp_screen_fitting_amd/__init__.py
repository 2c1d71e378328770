"""MI355X-native KL a-term screen fitter (drop-in for the KL path of
ska-sdp-screen-fitting).  Python host code over the C ABI of libscreenfit.so
(hand-written HIP for gfx950); see DESIGN.md."""

from ._lib import (Context, ScreenFitError, get_context, load_library,  # noqa: F401
                   private_context)

__version__ = "0.1.0"


def make_aterm_image(*args, **kwargs):
    """See :func:`ska_sdp_screen_fitting_amd.make_aterm_images.make_aterm_image`."""
    from .make_aterm_images import make_aterm_image as _impl
    return _impl(*args, **kwargs)
