"""VAESNe — MI355X-native (gfx950) build of the VAESNe multimodal-VAE training step.

Drop-in for the reference package's hot path (module paths, class names,
constructor kwargs and state_dict keys of YunyiShen/VAESNe-dev
package/VAESNe): PhotometricVAE, SpectraVAE, photospecMMVAE, losses.elbo /
m_iwae / _m_iwae, training_util.training_step, data_util.multimodalDataset.
Every forward/backward op runs as a hand-written HIP kernel from
libvaesne_hip.so (include/vaesne_hip.h); there is no CPU path.
"""
