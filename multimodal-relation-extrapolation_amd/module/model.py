"""UnifiedModel (module/model.py:517-686) on this build's kernels, and the text branch of its
frozen M3AE encoder (MaskedMultimodalAutoencoder, model.py:200-356).

* `UnifiedModel(args, hidden_channels, dataset, num_relations, noise_dim)` keeps the reference
  constructor and module names, so its state-dict keys are the reference's:
  generate_fc_layer / des_rel_map_layer1 / des_rel_map_layer2 .{weight_orig, weight_u,
  weight_v, bias} (spectral_norm.py:129-137), layer_norm.{a_2, b_2}, M3AEmodel.* -- each once.
* `generate(description_tokens, des_padding_mask, noise)` (model.py:674-686): the HIP M3AE
  text encoder (csrc/m3ae.hip) -> the fused spectral-norm MLP + LayerNormalization
  (csrc/generator.hip). `generator` is that MLP as an mmre.generator.RelationGenerator view
  sharing the same layers (not a registered submodule: no duplicate keys); ZSLmodule's GAN step
  trains it.
* `forward_relation_emb` (model.py:599-610): encoder CLS -> des_rel_map_layer1 ->
  des_rel_map_layer2 on the HIP spectral-norm weight + split-K GEMM (differentiable), and the
  LayerNormalization computed and discarded exactly as the reference does (:609).
* `forward(edge_index, edge_type, batch)` (model.py:612-669): the entity representations x_gcn
  come from M3AE's image/text branch + the RGCN encoder, which are outside this build's path
  (SURVEY.md §2 row 15); the caller supplies them as batch['x_gcn'] (main.py here: a trainable
  structure table). The relation side runs as above; the masked-autoencoder outputs are absent.
* Reference checkpoints load with strict=True: tensors of the out-of-path parts (RGCN `conv.*`,
  `node_embedding.*`, M3AE's image embedding / decoder / mask embeddings) are accepted, carried
  unchanged and written back by state_dict(), never computed with.
"""
from types import SimpleNamespace

import torch
import torch.nn as nn

from mmre._lib import MMREError
from mmre.generator import RelationGenerator
from mmre.m3ae import M3AETextEncoder


class _CarriesOutOfPath:
    """Mixin for modules whose reference counterpart holds parameters this build does not
    compute: state-dict entries under OUT_OF_PATH names are kept as opaque tensors on load and
    emitted again by state_dict()."""

    OUT_OF_PATH = ()

    def _init_carry(self):
        object.__setattr__(self, "_carried", {})
        self._register_state_dict_hook(_emit_carried)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)
        for k in list(state_dict.keys()):
            if not k.startswith(prefix):
                continue
            rest = k[len(prefix):]
            if rest.split(".", 1)[0] in self.OUT_OF_PATH:
                self._carried[rest] = state_dict[k].detach().clone()
                if k in unexpected_keys:
                    unexpected_keys.remove(k)


def _emit_carried(module, state_dict, prefix, local_metadata):
    for k, v in module._carried.items():
        state_dict[prefix + k] = v
    return state_dict


class MaskedMultimodalAutoencoder(_CarriesOutOfPath, M3AETextEncoder):
    """Text branch of the reference's MaskedMultimodalAutoencoder with its constructor
    (model.py:229): config_updates' model_type picks the size (utils.py:126-192, default
    'small': d 384, 12 blocks, 6 heads). forward_representation(image=None, text,
    text_padding_mask, deterministic=True) returns (cls_x (B, 1, D), None). The image branch,
    the masked-autoencoder decoder and their parameters are outside this path (carried in
    state dicts, never computed)."""

    OUT_OF_PATH = ("image_embedding", "encoder_image_type_embedding", "decoder_image_type_embedding",
                   "decoder_text_type_embedding", "image_mask_embedding", "text_mask_embedding", "decoder",
                   "decoder_input_projection", "decoder_image_output", "decoder_text_output")

    def __init__(self, text_vocab_size, patch_size=16, image_output_dim=768, config_updates=None):
        cfg = dict(config_updates or {})
        super().__init__(text_vocab_size, model_type=cfg.get("model_type", "small") or "small")
        self.patch_size = patch_size
        self.image_output_dim = image_output_dim
        self.config = SimpleNamespace(**dict(cfg, emb_dim=self.emb_dim, depth=self.depth, num_heads=self.num_heads))
        self._init_carry()


class UnifiedModel(_CarriesOutOfPath, nn.Module):
    OUT_OF_PATH = ("conv", "node_embedding")

    def __init__(self, args, hidden_channels, dataset, num_relations, noise_dim):
        super().__init__()
        image_output_dim = args.patch_size * args.patch_size * 3
        self.M3AEmodel = MaskedMultimodalAutoencoder(
            text_vocab_size=dataset.vocab_size, patch_size=args.patch_size, image_output_dim=image_output_dim,
            config_updates=dict(model_type=args.model_type, image_mask_ratio=args.image_mask_ratio,
                                text_mask_ratio=args.text_mask_ratio))
        self.is_evaluate = args.evaluate
        self.patch_size = args.patch_size
        cfg = dataset.config
        self.is_contrastive = not (args.contrastive_loss_weight == 0.0 or cfg.image_only or cfg.text_only)
        self.paired_tokenizer_max_length = cfg.tokenizer_max_length
        self.token_num = cfg.unpaired_tokenizer_max_length
        self.num_relations = num_relations
        self.num_nodes = dataset.num_nodes
        self.reduced_dim = self.M3AEmodel.emb_dim
        self.dim = args.emb_dim
        self.noise_dim = noise_dim
        self.hidden_channels = hidden_channels
        gen = RelationGenerator(self.reduced_dim, noise_dim, self.dim)
        self.des_rel_map_layer1 = gen.des_rel_map_layer1   # 384 -> 200 (model.py:544-545)
        self.des_rel_map_layer2 = gen.des_rel_map_layer2   # 200 -> 200 (:546-547)
        self.generate_fc_layer = gen.generate_fc_layer     # 399 -> 384 (:548-549)
        self.layer_norm = gen.layer_norm                   # (:555)
        object.__setattr__(self, "generator", gen)         # shares the layers above; not a submodule
        self._init_carry()

    def get_model_device(self):
        return next(self.parameters()).device

    def set_evaluate(self, flag: bool):
        self.is_evaluate = flag

    def _cls(self, description_tokens, des_padding_mask):
        with torch.no_grad():
            cls, _ = self.M3AEmodel.forward_representation(image=None, text=description_tokens,
                                                           text_padding_mask=des_padding_mask, deterministic=True)
        return cls.reshape(cls.shape[0], -1)

    def forward_relation_emb(self, description_tokens, des_padding_mask):
        """model.py:599-610: CLS -> des_rel_map_layer1 -> des_rel_map_layer2; the
        LayerNormalization output is computed and discarded, as in the reference (:609)."""
        from mmre.gemm import sn_linear
        rel_emb = self._cls(description_tokens, des_padding_mask)
        rel_emb = sn_linear(self.des_rel_map_layer1, rel_emb)
        rel_emb = sn_linear(self.des_rel_map_layer2, rel_emb)
        self.layer_norm(rel_emb)
        return rel_emb

    def forward(self, edge_index, edge_type, batch, deterministic=False):
        x_gcn = batch.get("x_gcn") if isinstance(batch, dict) else None
        if x_gcn is None:
            raise MMREError("UnifiedModel.forward: the entity encoder (M3AE image/text branch + RGCN, model.py:624-628) "
                            "is outside this build's path -- supply the entity representations as batch['x_gcn']")
        rel_emb = self.forward_relation_emb(batch["rel_des"], batch["rel_des_padding_mask"])
        if self.is_evaluate:
            return x_gcn, rel_emb
        batch_output = dict(image_output=None, text_output=None, image_mask=None, text_mask=None,
                            contrastive_loss=0.0)
        return x_gcn, rel_emb, batch_output

    def generate_from_cls(self, cls, noise):
        """generate() after the encoder (model.py:679-686), for precomputed CLS rows."""
        self.generator.train(self.training)
        return self.generator(cls, noise)

    def generate(self, description_tokens, des_padding_mask, noise):
        return self.generate_from_cls(self._cls(description_tokens, des_padding_mask), noise)
