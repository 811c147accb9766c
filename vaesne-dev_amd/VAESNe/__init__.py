"""VAESNe — MI355X-native (gfx950) build of the VAESNe multimodal-VAE training step.

Drop-in for the reference package's hot path (module paths, class names,
constructor kwargs and state_dict keys of YunyiShen/VAESNe-dev
package/VAESNe): PhotometricVAE, SpectraVAE, photospecMMVAE, losses.elbo /
m_iwae / _m_iwae, training_util.training_step, data_util.multimodalDataset.
Every forward/backward op runs as a hand-written HIP kernel from
libvaesne_hip.so (include/vaesne_hip.h); there is no CPU path for these models.
(ImageVAE.HostImgVAE, BASELINE config 1, is the reference's host-only image VAE and
runs PyTorch host ops: SURVEY.md §8(a) a16.)

Launched one process per GPU (torchrun sets LOCAL_RANK), importing the package
selects this rank's GPU, so a script's `.to('cuda')` lands on it with the script
unchanged; training_step then brings up the RCCL process group (distributed.py).
"""
import os as _os


def _select_local_gpu():
    if int(_os.environ.get("WORLD_SIZE", "1") or 1) <= 1 or "LOCAL_RANK" not in _os.environ:
        return
    import torch
    if torch.cuda.is_available():
        # more ranks than GPUs (VAESNE_DP_BACKEND=gloo rehearsals): ranks share them
        torch.cuda.set_device(int(_os.environ["LOCAL_RANK"]) % max(1, torch.cuda.device_count()))


_select_local_gpu()
