"""Zero-shot GAN training step (ZSLmodule.train, module/zsl_module.py:350-600) on one GPU.

Per step the reference runs, for a batch of (relation description, real pair, false pair)
rows: Extractor vectors of the real and false pairs, the generator on the relation's CLS +
noise, the spectral-normalised Discriminator (zsl_module.py:112-138) three or four times,
the WGAN-GP gradient penalty (module/utils.py:692-707, a double backward), the losses and an
Adam step -- about two hundred small launches, far below one MI355X's width at N = 512 rows.
Here:
  * Extractor vectors: the fused HIP encode over per-entity tables built once (the Extractor
    is frozen during GAN training; mmre.extractor);
  * generator forward + backward: HIP (mmre_generator_forward_save / _backward, spectral-norm
    chain rule included);
  * Discriminator, gradient penalty and Adam: autograd on the device with the Discriminator's
    pieces on HIP (mmre.gemm): every matrix product and its derivatives (the penalty's double
    backward included) on the split-K GEMM -- a library GEMM ran each of these 200-512-sided
    products on one workgroup -- the spectral-norm weight in one launch, LayerNormalization;
  * each D step and G step is captured once into a hipGraph (torch.cuda.CUDAGraph on ROCm)
    over static input buffers and replayed: one graph launch per step instead of ~200 kernel
    launches. Noise and the GP's alpha are drawn inside the graph (graph-safe Philox).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .extractor import encode
from .gemm import mm


def _cls_scores(class_scores, labels):
    return class_scores.gather(1, labels.view(-1, 1)).squeeze(1)


class ZSLGANStep:
    """generator: mmre.generator.RelationGenerator (the reference's generate_model MLP);
    discriminator: module.zsl_module.Discriminator; cls_table (n_rel_ids, reduced_dim): the
    frozen encoder's CLS of every relation description; centroids (n_train_rel, d)
    (zsl_module.py:371-383); ranker: mmre.extractor.ZSLRanker over the entity graph (its
    tables give the Extractor vectors of (head, tail) entity-id pairs)."""

    def __init__(self, generator, discriminator, cls_table, centroids, ranker, lr_G=1e-4, lr_D=1e-4,
                 pretrain_margin=5.0, gan_batch_rela=2, gp_lambda=10.0, vecs_fn=None):
        self.G, self.D = generator, discriminator
        self.cls_table, self.centroids, self.ranker = cls_table, centroids, ranker
        self.margin, self.gan_batch_rela, self.gp_lambda = float(pretrain_margin), int(gan_batch_rela), gp_lambda
        self.n_labels = int(centroids.shape[0])
        # vecs_fn(heads, tails): Extractor vectors of a training-mode Extractor (dropout,
        # mmre.extractor_train.PretrainStep.vectors); None: the frozen eval-mode tables
        self.vecs_fn = vecs_fn
        dev = cls_table.device
        self.optim_D = torch.optim.Adam([p for p in self.D.parameters() if p.requires_grad], lr=lr_D,
                                        betas=(0.5, 0.9), capturable=True)
        self.optim_G = torch.optim.Adam([p for p in self.G._params() if p.requires_grad], lr=lr_G,
                                        betas=(0.5, 0.9), capturable=True)
        self.device = dev
        self.keep_grads = False  # tests: copy the gradients before each optimiser step
        self._graphs = {}
        self._static = {}

    # ---------------------------------------------------------------- pieces
    def extractor_vecs(self, heads, tails):
        if self.vecs_fn is not None:
            return self.vecs_fn(heads, tails)
        r = self.ranker
        g, _ = encode(r.pack, r.dim, r.ln_eps, r.left, heads, r.right, tails, want_g=True, want_score=False)
        return g

    def gradient_penalty(self, real, fake, alpha):
        """calc_gradient_penalty (module/utils.py:692-707) with alpha (N, 1) given."""
        inter = (alpha * real + (1 - alpha) * fake).requires_grad_(True)
        _, disc, _ = self.D(inter, self.centroids)
        grads = torch.autograd.grad(outputs=disc, inputs=inter, grad_outputs=torch.ones_like(disc),
                                    create_graph=True, retain_graph=True, only_inputs=True)[0]
        return ((grads.norm(2, dim=1) - 1) ** 2).mean() * self.gp_lambda

    # ---------------------------------------------------------------- steps
    def d_step(self, rel, q_head, q_tail, f_head, f_tail, labels, noise, alpha):
        """One Discriminator step (zsl_module.py:419-509). Returns the five logged losses."""
        self.D.train()
        self.G.eval()
        real = self.extractor_vecs(q_head, q_tail)
        neg = self.extractor_vecs(f_head, f_tail)
        with torch.no_grad():
            fake = self.G(self.cls_table.index_select(0, rel), noise)
        _, real_dec, real_cls = self.D(real, self.centroids)
        _, fake_dec, fake_cls = self.D(fake, self.centroids)
        _, _, neg_cls = self.D(neg, self.centroids)
        loss_real = -torch.mean(real_dec)
        loss_fake = torch.mean(fake_dec)
        neg_s = _cls_scores(neg_cls, labels)
        loss_rela = F.relu(self.margin - (_cls_scores(real_cls, labels) - neg_s)).mean()
        loss_fake_cls = F.relu(self.margin - (_cls_scores(fake_cls, labels) - neg_s)).mean()
        gp = self.gradient_penalty(real, fake, alpha)
        loss = loss_real + 0.5 * loss_rela + loss_fake + gp + 0.5 * loss_fake_cls
        loss.backward()
        if self.keep_grads:
            self.grads_d = [p.grad.detach().clone() for p in self.D.parameters() if p.requires_grad]
        self.optim_D.step()
        self.optim_D.zero_grad(set_to_none=False)
        self.G.zero_grad(set_to_none=False)
        return torch.stack([loss.detach(), loss_real.detach(), loss_rela.detach(), loss_fake.detach(),
                            loss_fake_cls.detach()])

    def g_step(self, rel, q_head, q_tail, f_head, f_tail, labels, noise):
        """One Generator step (zsl_module.py:511-600). Returns loss_G and its parts. The
        Discriminator's parameter gradients of loss_G, which the reference computes and then
        clears (Discriminator.zero_grad(), zsl_module.py:600), are not computed."""
        frozen = [p for p in self.D.parameters() if p.requires_grad]
        for p in frozen:
            p.requires_grad_(False)
        try:
            return self._g_step(rel, q_head, q_tail, f_head, f_tail, labels, noise)
        finally:
            for p in frozen:
                p.requires_grad_(True)

    def _g_step(self, rel, q_head, q_tail, f_head, f_tail, labels, noise):
        self.D.eval()
        self.G.train()
        sample = self.G(self.cls_table.index_select(0, rel), noise)
        real = self.extractor_vecs(q_head, q_tail)
        neg = self.extractor_vecs(f_head, f_tail)
        _, dec, cls = self.D(sample, self.centroids)
        _, _, real_cls = self.D(real, self.centroids)
        _, _, neg_cls = self.D(neg, self.centroids)
        loss_fake = -torch.mean(dec)
        neg_s = _cls_scores(neg_cls, labels)
        loss_cls = F.relu(self.margin - (_cls_scores(cls, labels) - neg_s)).mean()
        loss_real_cls = F.relu(self.margin - (_cls_scores(real_cls, labels) - neg_s)).mean()
        # visual pivot regularisation (zsl_module.py:564-581): per label present in the batch,
        # |mean(sample rows of the label) - centroid|_2, summed, / gan_batch_rela
        onehot = F.one_hot(labels, self.n_labels).to(sample.dtype)          # (N, L)
        cnt = onehot.sum(0)                                                  # (L,)
        means = mm(onehot.t(), sample) / cnt.clamp(min=1).unsqueeze(1)       # (L, d)
        dist = ((means - self.centroids) ** 2).sum(1).sqrt()
        loss_vp = torch.where(cnt > 0, dist, torch.zeros_like(dist)).sum() * (1.0 / self.gan_batch_rela)
        loss = loss_fake + loss_cls + 3.0 * loss_vp
        loss.backward()
        if self.keep_grads:
            self.grads_g = [p.grad.detach().clone() for p in self.G._params()]
        self.optim_G.step()
        self.G.zero_grad(set_to_none=False)
        self.D.zero_grad(set_to_none=False)
        return torch.stack([loss.detach(), loss_fake.detach(), loss_cls.detach(), loss_real_cls.detach(),
                            loss_vp.detach()])

    # ---------------------------------------------------------------- hipGraph replay
    def _buffers(self, n):
        if n not in self._static:
            dev = self.device
            li = lambda: torch.zeros(n, dtype=torch.int64, device=dev)
            self._static[n] = dict(rel=li(), q_head=li(), q_tail=li(), f_head=li(), f_tail=li(), labels=li(),
                                   noise=torch.zeros((n, self.G.noise_dim), device=dev),
                                   alpha=torch.zeros((n, 1), device=dev))
        return self._static[n]

    def _capture(self, kind, n, draw):
        b = self._buffers(n)

        def body():
            if draw:  # graph-safe RNG: fresh noise / alpha at every replay (torch.randn / torch.rand)
                b["noise"].normal_()
                b["alpha"].uniform_()
            if kind == "d":
                return self.d_step(b["rel"], b["q_head"], b["q_tail"], b["f_head"], b["f_tail"], b["labels"],
                                   b["noise"], b["alpha"])
            return self.g_step(b["rel"], b["q_head"], b["q_tail"], b["f_head"], b["f_tail"], b["labels"], b["noise"])

        # the first call is a real step run eagerly on a side stream: it is the warm-up the
        # capture needs (allocator pools, .grad tensors, Adam state); the capture that follows
        # records the step without running it
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):
            first = body()
        torch.cuda.current_stream(self.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = body()
        self._graphs[(kind, n, draw)] = (g, out)
        return first

    def replay(self, kind, batch, draw=True):
        """Run a D ('d') or G ('g') step on `batch` (dict of device tensors: rel, q_head, q_tail,
        f_head, f_tail, labels [, noise, alpha]) from its hipGraph; noise / alpha are drawn in the
        graph when draw. The first call per (kind, batch size, draw) runs the step eagerly and
        captures it; later calls replay. The returned loss tensor is the graph's static output
        (overwritten by the next replay)."""
        n = int(batch["q_head"].shape[0])
        b = self._buffers(n)
        for k, v in batch.items():
            b[k].copy_(v, non_blocking=True)
        key = (kind, n, draw)
        if key not in self._graphs:
            return self._capture(kind, n, draw)
        g, out = self._graphs[key]
        g.replay()
        return out
