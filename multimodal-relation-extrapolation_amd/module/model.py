"""The relation-embedding generator of UnifiedModel (module/model.py:517-686).

`UnifiedModelGenerator.generate(description_tokens, des_padding_mask, noise)` keeps the reference
signature (model.py:674). The frozen M3AE text encoder that turns the description tokens into
the (N, 384) CLS vector (model.py:675-678) is upstream of the hot path; pass it as `encoder`
(any callable tokens, mask -> CLS) or call `generate_from_cls(cls, noise)` directly. The
spectral-normalised MLP + LayerNormalization run as one HIP launch pair (csrc/generator.hip).
State-dict names follow the reference: generate_fc_layer / des_rel_map_layer1 /
des_rel_map_layer2 .{weight_orig, weight_u, weight_v, bias}, layer_norm.{a_2, b_2}."""
import torch
import torch.nn as nn

from mmre.generator import RelationGenerator


class UnifiedModelGenerator(nn.Module):
    def __init__(self, emb_dim=200, noise_dim=15, reduced_dim=384, num_relations=None, encoder=None):
        super().__init__()
        self.dim = emb_dim
        self.noise_dim = noise_dim
        self.reduced_dim = reduced_dim
        self.num_relations = num_relations
        self.encoder = encoder
        self.gen = RelationGenerator(reduced_dim, noise_dim, emb_dim)
        # reference names
        self.generate_fc_layer = self.gen.generate_fc_layer
        self.des_rel_map_layer1 = self.gen.des_rel_map_layer1
        self.des_rel_map_layer2 = self.gen.des_rel_map_layer2

    @property
    def layer_norm_params(self):
        return self.gen.ln_a, self.gen.ln_b

    def generate_from_cls(self, cls, noise):
        self.gen.train(self.training)
        return self.gen(cls, noise)

    def generate(self, description_tokens, des_padding_mask, noise):
        if self.encoder is None:
            raise RuntimeError("UnifiedModelGenerator.generate needs the frozen text encoder (M3AE, out of the "
                               "hot path); pass encoder=... or call generate_from_cls(cls, noise)")
        with torch.no_grad():
            cls = self.encoder(description_tokens, des_padding_mask)
        return self.generate_from_cls(cls.reshape(cls.shape[0], -1), noise)
