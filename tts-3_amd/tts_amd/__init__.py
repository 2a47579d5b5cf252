"""tts_amd — MI355X-native (gfx950) mel->waveform path for Coqui TTS.

Drop-in replacements, backed by ``libtts_mi355x.so`` (include/tts_mi355x.h):

* ``tts_amd.vocoder.HifiganGenerator``  for TTS.vocoder.models.hifigan_generator.HifiganGenerator
* ``tts_amd.vocoder.GAN``               the inference surface of TTS.vocoder.models.gan.GAN
* ``tts_amd.tts.Decoder``               for TTS.tts.layers.glow_tts.decoder.Decoder (reverse)
"""
__version__ = "0.1.0"
