"""The helpers of module/utils.py that sit on this build's path.

* set_random_seed (utils.py:232-236): torch / cuda / numpy seeds; like the reference it does not
  seed Python's `random` (P13).
* weights_init (utils.py:119-123): xavier_normal_ weights, zero biases for every *Linear*.
* generate_rel_embed (utils.py:529-546): the 'seen' relation table of ZSLmodule.update_embed =
  UnifiedModel.forward_relation_emb over every relation description (HIP M3AE text encoder +
  spectral-norm layers). 'unseen' needs the DistillModel (module/DistillModel.py, unused by the
  reference's main.py and outside this path) and raises.
* generate_ent_embed (utils.py:479-527) is M3AE's image/text branch + the RGCN encoder over all
  entities, outside this path; here it returns the table of the structure encoder that stands
  in for them (main.py attaches it to the strategy as `ent_encoder`) and raises without one.
"""
import numpy as np
import torch

from mmre._lib import MMREError


def set_random_seed(seed):
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)


def weights_init(m):
    if "Linear" in m.__class__.__name__:
        torch.nn.init.xavier_normal_(m.weight.data)
        torch.nn.init.constant_(m.bias, 0.0)


def generate_rel_embed(dataset, model, d_model, device, rel_type="unseen"):
    """(num_relations, emb_dim) CPU tensor. model: the NegativeSampling strategy holding the
    UnifiedModel as .model (main.py:207-208)."""
    um = model.model
    rel_list = torch.arange(0, um.num_relations)
    batch_data = dataset.generate_batch([], rel_list)
    if rel_type == "seen":
        with torch.no_grad():
            rel_embs = um.forward_relation_emb(description_tokens=batch_data["rel_des"].to(device),
                                               des_padding_mask=batch_data["rel_des_padding_mask"].to(device))
    elif rel_type == "unseen":
        if d_model is None:
            raise MMREError("generate_rel_embed('unseen') needs the DistillModel (module/DistillModel.py), "
                            "outside this build's path")
        with torch.no_grad():
            rel_embs = d_model.predict(batch_data["rel_des"].to(device))
    else:
        raise ValueError(f"rel_type must be 'seen' or 'unseen', not {rel_type!r}")
    return rel_embs.cpu()


def generate_ent_embed(args, dataset, model, device):
    """(num_nodes, emb_dim) CPU tensor of entity representations (see the module docstring)."""
    enc = getattr(model, "ent_encoder", None)
    if enc is None:
        raise MMREError("generate_ent_embed: the multimodal entity encoder (M3AE image/text + RGCN, "
                        "utils.py:479-527) is outside this build's path; attach a structure encoder as "
                        "model.ent_encoder (main.py does)")
    return enc.weight.detach().cpu().clone()
