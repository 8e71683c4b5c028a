"""adaptsegnet_amd — MI355X-native AdaptSegNet adversarial-training hot path.

Drop-in modules for the reference call sites of train_gta2cityscapes_multi.py:
  adaptsegnet_amd.model.DeeplabMulti, adaptsegnet_amd.model.FCDiscriminator,
  adaptsegnet_amd.utils.loss.CrossEntropy2d, adaptsegnet_amd.functional (softmax, losses),
  adaptsegnet_amd.optim (fused SGD / Adam over the parameter arenas),
  adaptsegnet_amd.train (the single-/multi-level adversarial step).
All arithmetic runs in libadaptseg.so (hand-written HIP for gfx950); see include/adaptseg.h.
"""
__version__ = "0.1.0"
