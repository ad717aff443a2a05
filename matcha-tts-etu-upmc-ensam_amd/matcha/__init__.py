"""MI355X-native Matcha-TTS training hot path.

Drop-in for the reference package layout (``matcha.models.matcha_tts.MatchaTTS``,
``matcha.models.components.{decoder,flow_matching,transformer,text_encoder}``,
``matcha.utils.monotonic_align.maximum_path``, ``matcha.utils.model``): put the directory that holds
this package first on ``sys.path``.  Device compute runs in ``lib/libmtts_hip.so`` (gfx950 HIP,
C ABI in ``include/mtts.h``), loaded by :mod:`matcha._native`.
"""
__version__ = "0.1.0"
