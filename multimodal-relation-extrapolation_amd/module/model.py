"""The relation-embedding generator of UnifiedModel (module/model.py:517-686) and the text
branch of its frozen M3AE encoder (model.py:200-356).

`UnifiedModelGenerator.generate(description_tokens, des_padding_mask, noise)` keeps the reference
signature (model.py:674). The frozen M3AE text encoder that turns the description tokens into
the (N, 384) CLS vector (model.py:675-678) is `M3AEmodel` (the reference attribute name; pass it
as `encoder=`, e.g. a `MaskedMultimodalAutoencoder` below, csrc/m3ae.hip), or call
`generate_from_cls(cls, noise)` directly. The spectral-normalised MLP + LayerNormalization run as
one HIP launch pair (csrc/generator.hip). State-dict names follow the reference:
generate_fc_layer / des_rel_map_layer1 / des_rel_map_layer2 .{weight_orig, weight_u, weight_v,
bias}, layer_norm.{a_2, b_2}, M3AEmodel.{text_embedding, cls_token, encoder.blocks.*, ...}."""
import torch
import torch.nn as nn

from mmre.generator import RelationGenerator
from mmre.m3ae import M3AETextEncoder


class MaskedMultimodalAutoencoder(M3AETextEncoder):
    """Text branch of the reference's MaskedMultimodalAutoencoder with its constructor
    (model.py:229): config_updates' model_type picks the size (utils.py:126-192, default
    'small': d 384, 12 blocks, 6 heads). forward_representation(image=None, text,
    text_padding_mask, deterministic=True) returns (cls_x (B, 1, D), None); the image branch,
    the masked-autoencoder decoder and its losses are outside this path."""

    def __init__(self, text_vocab_size, patch_size=16, image_output_dim=768, config_updates=None):
        cfg = dict(config_updates or {})
        super().__init__(text_vocab_size, model_type=cfg.get("model_type", "small") or "small")
        self.patch_size = patch_size
        self.image_output_dim = image_output_dim


class UnifiedModelGenerator(nn.Module):
    def __init__(self, emb_dim=200, noise_dim=15, reduced_dim=384, num_relations=None, encoder=None):
        super().__init__()
        self.dim = emb_dim
        self.noise_dim = noise_dim
        self.reduced_dim = reduced_dim
        self.num_relations = num_relations
        self.M3AEmodel = encoder  # model.py:521 (frozen text encoder: tokens, mask -> CLS)
        self.gen = RelationGenerator(reduced_dim, noise_dim, emb_dim)
        # reference names
        self.generate_fc_layer = self.gen.generate_fc_layer
        self.des_rel_map_layer1 = self.gen.des_rel_map_layer1
        self.des_rel_map_layer2 = self.gen.des_rel_map_layer2

    @property
    def encoder(self):
        return self.M3AEmodel

    @property
    def layer_norm_params(self):
        return self.gen.ln_a, self.gen.ln_b

    def generate_from_cls(self, cls, noise):
        self.gen.train(self.training)
        return self.gen(cls, noise)

    def generate(self, description_tokens, des_padding_mask, noise):
        enc = self.M3AEmodel
        if enc is None:
            raise RuntimeError("UnifiedModelGenerator.generate needs the frozen text encoder (M3AE); pass "
                               "encoder=MaskedMultimodalAutoencoder(...) or call generate_from_cls(cls, noise)")
        with torch.no_grad():
            if hasattr(enc, "forward_representation"):
                cls, _ = enc.forward_representation(image=None, text=description_tokens,
                                                    text_padding_mask=des_padding_mask, deterministic=True)
            else:
                cls = enc(description_tokens, des_padding_mask)
        return self.generate_from_cls(cls.reshape(cls.shape[0], -1), noise)
