"""ViT-B/16 built from the drop-in approx operators (BASELINE config 4 as a whole model).

The float network has the module tree and parameter names of the HF ``ViTForImageClassification``
the reference wraps (vit.embeddings.{cls_token, position_embeddings, patch_embeddings.projection},
vit.encoder.layer[i].{attention.attention.{query,key,value}, attention.output.dense,
intermediate.dense, output.dense, layernorm_before, layernorm_after}, vit.layernorm, classifier),
so a ``google/vit-base-patch16-224`` state dict loads with ``load_float_weights``; it is written
in plain torch because the checkpoint needs the network and the installed transformers release
no longer has the module classes (ViTSdpaAttention, ViTIntermediate, ...) the reference's
specials are keyed on.  QuantizedVisionTransformerForImageClassification wraps it the way
models/vit_quantized_approx.py:19-398 does: every Linear becomes a QCustomLinearTorch and every
LayerNorm a QuantLayerNorm through ``quantize_model``, the patch projection an exact
QCustomConv2dTorch, and the activation quantizers sit where the reference's Quantized* modules
put them (embeddings, attention context, first residual, MLP activation, second residual,
encoder output).

Extension over the reference: its encoder linears receive [B, 197, 768] inputs and fail the
2-D assertion of custom_matmul_vectorize under approx_flag; here every approx linear
of the model folds the leading dims into rows (``flatten_leading_dims``), so each token row gets
exactly the approx product the reference computes for a 2-D input.  Attention (softmax(QK^T)V)
is the reference's plain fp32 SDPA (vit_quantized_approx.py:188-196), not an approx product.
"""
import torch
import torch.nn.functional as F
from torch import nn

from .approx_calculation import QCustomLinearTorch
from .model_wrap import QuantizedModel, fused_linear_tail, quantize_model
from .quantization.base_quantized_classes import QuantizedActivation


# ------------------------------------------------------------------------- float ViT (HF layout)
class ViTPatchEmbeddings(nn.Module):
    def __init__(self, image_size, patch_size, num_channels, hidden):
        super().__init__()
        self.image_size = (image_size, image_size)
        self.patch_size = (patch_size, patch_size)
        self.num_channels = num_channels
        self.num_patches = (image_size // patch_size) ** 2
        self.projection = nn.Conv2d(num_channels, hidden, patch_size, patch_size)

    def forward(self, x):
        return self.projection(x).flatten(2).transpose(1, 2)


class ViTEmbeddings(nn.Module):
    def __init__(self, image_size, patch_size, num_channels, hidden, dropout):
        super().__init__()
        self.patch_embeddings = ViTPatchEmbeddings(image_size, patch_size, num_channels, hidden)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, hidden))
        self.position_embeddings = nn.Parameter(torch.zeros(1, self.patch_embeddings.num_patches + 1, hidden))
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        e = self.patch_embeddings(x)
        e = torch.cat((self.cls_token.expand(x.shape[0], -1, -1), e), dim=1) + self.position_embeddings
        return self.dropout(e)


class ViTSelfAttention(nn.Module):
    def __init__(self, hidden, heads, dropout):
        super().__init__()
        self.num_attention_heads = heads
        self.attention_head_size = hidden // heads
        self.all_head_size = hidden
        self.query = nn.Linear(hidden, hidden)
        self.key = nn.Linear(hidden, hidden)
        self.value = nn.Linear(hidden, hidden)
        self.dropout = nn.Dropout(dropout)
        self.attention_probs_dropout_prob = dropout

    def forward(self, x):
        return _attention(self, x)


class ViTSelfOutput(nn.Module):
    def __init__(self, hidden, dropout):
        super().__init__()
        self.dense = nn.Linear(hidden, hidden)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        return self.dropout(self.dense(x))


class ViTAttention(nn.Module):
    def __init__(self, hidden, heads, dropout):
        super().__init__()
        self.attention = ViTSelfAttention(hidden, heads, dropout)
        self.output = ViTSelfOutput(hidden, dropout)

    def forward(self, x):
        return self.output(self.attention(x))


class ViTIntermediate(nn.Module):
    def __init__(self, hidden, mlp):
        super().__init__()
        self.dense = nn.Linear(hidden, mlp)
        self.intermediate_act_fn = nn.GELU()

    def forward(self, x):
        return self.intermediate_act_fn(self.dense(x))


class ViTOutput(nn.Module):
    def __init__(self, hidden, mlp, dropout):
        super().__init__()
        self.dense = nn.Linear(mlp, hidden)
        self.dropout = nn.Dropout(dropout)

    def forward(self, h, input_tensor):
        return self.dropout(self.dense(h)) + input_tensor


class ViTLayer(nn.Module):
    def __init__(self, hidden, heads, mlp, dropout, eps):
        super().__init__()
        self.attention = ViTAttention(hidden, heads, dropout)
        self.intermediate = ViTIntermediate(hidden, mlp)
        self.output = ViTOutput(hidden, mlp, dropout)
        self.layernorm_before = nn.LayerNorm(hidden, eps=eps)
        self.layernorm_after = nn.LayerNorm(hidden, eps=eps)

    def forward(self, h):
        h = self.attention(self.layernorm_before(h)) + h
        return self.output(self.intermediate(self.layernorm_after(h)), h)


class ViTEncoder(nn.Module):
    def __init__(self, layers, *args):
        super().__init__()
        self.layer = nn.ModuleList([ViTLayer(*args) for _ in range(layers)])
        self.gradient_checkpointing = False

    def forward(self, h):
        for lay in self.layer:
            h = lay(h)
        return h


class ViTModel(nn.Module):
    def __init__(self, image_size, patch_size, num_channels, hidden, layers, heads, mlp, dropout, eps):
        super().__init__()
        self.embeddings = ViTEmbeddings(image_size, patch_size, num_channels, hidden, dropout)
        self.encoder = ViTEncoder(layers, hidden, heads, mlp, dropout, eps)
        self.layernorm = nn.LayerNorm(hidden, eps=eps)

    def forward(self, x):
        return self.layernorm(self.encoder(self.embeddings(x)))


class ViTForImageClassification(nn.Module):
    """google/vit-base-patch16-224 by default (hidden 768, 12 layers, 12 heads, MLP 3072,
    LayerNorm eps 1e-12, 1000 classes), HF's initialisation (truncated normal, std 0.02)."""

    def __init__(self, image_size=224, patch_size=16, num_channels=3, hidden=768, layers=12, heads=12, mlp=3072,
                 num_labels=1000, dropout=0.0, eps=1e-12, init_std=0.02):
        super().__init__()
        self.vit = ViTModel(image_size, patch_size, num_channels, hidden, layers, heads, mlp, dropout, eps)
        self.classifier = nn.Linear(hidden, num_labels)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Conv2d)):
                nn.init.trunc_normal_(m.weight, std=init_std)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        nn.init.trunc_normal_(self.vit.embeddings.position_embeddings, std=init_std)
        nn.init.trunc_normal_(self.vit.embeddings.cls_token, std=init_std)

    def forward(self, x):
        return self.classifier(self.vit(x)[:, 0, :])


def _attention(mod, x):
    """softmax(Q K^T / sqrt(d)) V per head through torch's SDPA, as the reference's
    QuantizedViTSelfAttention.forward (vit_quantized_approx.py:181-199)."""
    def heads(t):
        return t.view(t.shape[:-1] + (mod.num_attention_heads, mod.attention_head_size)).permute(0, 2, 1, 3)
    q, k, v = heads(mod.query(x)), heads(mod.key(x)), heads(mod.value(x))
    ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=None,
                                         dropout_p=mod.attention_probs_dropout_prob if mod.training else 0.0,
                                         is_causal=False, scale=None)
    ctx = ctx.permute(0, 2, 1, 3).contiguous()
    return ctx.view(ctx.shape[:-2] + (mod.all_head_size,))


# ------------------------------------------------------------------------- quantized wrappers
class QuantizedVitPatchEmbeddings(QuantizedActivation):
    """vit_quantized_approx.py:56-83."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.projection = quantize_model(orig.projection, **quant_params)
        self.num_channels = orig.num_channels
        self.image_size = orig.image_size
        self.patch_size = orig.patch_size
        self.num_patches = orig.num_patches

    def forward(self, pixel_values, interpolate_pos_encoding=False):
        _, c, h, w = pixel_values.shape
        if c != self.num_channels:
            raise ValueError("Make sure that the channel dimension of the pixel values match with the one set in "
                             f"the configuration. Expected {self.num_channels} but got {c}.")
        if not interpolate_pos_encoding and (h, w) != tuple(self.image_size):
            raise ValueError(f"Input image size ({h}*{w}) doesn't match model ({self.image_size[0]}*"
                             f"{self.image_size[1]}).")
        return self.quantize_activations(self.projection(pixel_values).flatten(2).transpose(1, 2))


class QuantizedVitEmbeddings(QuantizedActivation):
    """vit_quantized_approx.py:85-115."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.patch_embeddings = quantize_model(orig.patch_embeddings,
                                               specials={ViTPatchEmbeddings: QuantizedVitPatchEmbeddings},
                                               **quant_params)
        self.cls_token = orig.cls_token
        self.position_embeddings = orig.position_embeddings
        self.dropout = orig.dropout

    def forward(self, x):
        e = self.patch_embeddings(x)
        e = torch.cat((self.cls_token.expand(x.shape[0], -1, -1), e), dim=1) + self.position_embeddings
        return self.quantize_activations(self.dropout(e))


class QuantizedViTImmediate(QuantizedActivation):
    """vit_quantized_approx.py:117-135 (the reference's spelling): dense, GELU, quantize."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.dense = quantize_model(orig.dense, **quant_params)
        self.intermediate_act_fn = orig.intermediate_act_fn

    def forward(self, h):
        act = self.intermediate_act_fn
        if isinstance(act, nn.GELU) and act.approximate == "none":  # dense + GELU + quantize: one launch
            fused = fused_linear_tail(self, self.dense, h, None, gelu=True)
            if fused is not None:
                return fused
        return self.quantize_activations(self.intermediate_act_fn(self.dense(h)))


class QuantizedViTOutput(QuantizedActivation):
    """vit_quantized_approx.py:137-156: dense, + residual, quantize."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.dense = quantize_model(orig.dense, **quant_params)
        self.dropout = orig.dropout

    def forward(self, h, input_tensor):
        fused = fused_linear_tail(self, self.dense, h, input_tensor, self.dropout)
        if fused is not None:
            return fused
        return self.quantize_activations(self.dropout(self.dense(h)) + input_tensor)


class QuantizedViTSelfAttention(QuantizedActivation):
    """vit_quantized_approx.py:159-199: approx Q / K / V, fp32 SDPA, quantized context."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.num_attention_heads = orig.num_attention_heads
        self.attention_head_size = orig.attention_head_size
        self.all_head_size = orig.all_head_size
        self.query = quantize_model(orig.query, **quant_params)
        self.key = quantize_model(orig.key, **quant_params)
        self.value = quantize_model(orig.value, **quant_params)
        self.dropout = orig.dropout
        self.training = orig.training
        self.attention_probs_dropout_prob = orig.attention_probs_dropout_prob

    def forward(self, x):
        return self.quantize_activations(_attention(self, x))


class QuantizedViTSelfOutput(QuantizedActivation):
    """vit_quantized_approx.py:202-217: dense only (its quantizer is unused, as in the reference)."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.dense = quantize_model(orig.dense, **quant_params)
        self.dropout = orig.dropout

    def forward(self, x):
        return self.dropout(self.dense(x))


class QuantizedViTSdpaAttention(QuantizedActivation):
    """vit_quantized_approx.py:219-240."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        specials = {ViTSelfAttention: QuantizedViTSelfAttention, ViTSelfOutput: QuantizedViTSelfOutput}
        self.attention = quantize_model(orig.attention, specials=specials, **quant_params)
        self.output = quantize_model(orig.output, specials=specials, **quant_params)

    def forward(self, x):
        return self.output(self.attention(x))


class QuantizedViTLayer(QuantizedActivation):
    """vit_quantized_approx.py:242-287: pre-LN attention, quantized first residual, pre-LN MLP
    whose output module adds and quantizes the second residual."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        specials = {ViTIntermediate: QuantizedViTImmediate, ViTOutput: QuantizedViTOutput,
                    ViTAttention: QuantizedViTSdpaAttention}
        self.intermediate = quantize_model(orig.intermediate, specials=specials, **quant_params)
        self.attention = quantize_model(orig.attention, specials=specials, **quant_params)
        self.output = quantize_model(orig.output, specials=specials, **quant_params)
        self.layernorm_before = quantize_model(orig.layernorm_before, **quant_params)
        self.layernorm_after = quantize_model(orig.layernorm_after, **quant_params)

    def forward(self, hidden_states, head_mask=None, output_attentions=False):
        att = self.attention
        ctx = att.attention(self.layernorm_before(hidden_states))
        h = fused_linear_tail(self, att.output.dense, ctx, hidden_states, att.output.dropout) \
            if isinstance(att, QuantizedViTSdpaAttention) and isinstance(att.output, QuantizedViTSelfOutput) else None
        if h is None:
            h = self.quantize_activations(att.output(ctx) + hidden_states)
        return self.output(self.intermediate(self.layernorm_after(h)), h)


class QuantizedViTEncoder(QuantizedActivation):
    """vit_quantized_approx.py:289-308."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        self.layer = quantize_model(orig.layer, specials={ViTLayer: QuantizedViTLayer}, **quant_params)
        self.gradient_checkpointing = orig.gradient_checkpointing

    def forward(self, hidden_states):
        for lay in self.layer:
            hidden_states = lay(hidden_states)
        return self.quantize_activations(hidden_states)


class QuantizedViTModel(QuantizedActivation):
    """vit_quantized_approx.py:330-364 (no pooler: the classification model has none)."""

    def __init__(self, orig, **quant_params):
        super().__init__(**quant_params)
        specials = {ViTEmbeddings: QuantizedVitEmbeddings, ViTEncoder: QuantizedViTEncoder}
        self.embeddings = quantize_model(orig.embeddings, specials=specials, **quant_params)
        self.encoder = quantize_model(orig.encoder, specials=specials, **quant_params)
        self.layernorm = quantize_model(orig.layernorm, **quant_params)

    def forward(self, x):
        return self.layernorm(self.encoder(self.embeddings(x)))


class QuantizedVisionTransformerForImageClassification(QuantizedModel):
    """vit_quantized_approx.py:367-391.  ``flatten_token_rows`` (default on) is the F4
    extension above; off, the encoder linears raise AssertionError like the reference's."""

    def __init__(self, model_fp, input_size=(1, 3, 224, 224), quant_setup=None, flatten_token_rows=True,
                 **quant_params):
        super().__init__(input_size)
        self.vit = quantize_model(model_fp.vit, specials={ViTModel: QuantizedViTModel}, **quant_params)
        self.classifier = quantize_model(model_fp.classifier, **quant_params)
        for m in self.modules():
            if isinstance(m, QCustomLinearTorch):
                m.flatten_leading_dims = flatten_token_rows

    def forward(self, x):
        return self.classifier(self.vit(x)[:, 0, :])


def vit_b16_approx(weights=None, image_size=224, patch_size=16, hidden=768, layers=12, heads=12, mlp=3072,
                   num_labels=1000, flatten_token_rows=True, seed=None, **cfg):
    """The reference's vit_quantized_approx (vit_quantized_approx.py:394-398) with random-init
    (or locally loaded) weights instead of ``from_pretrained``."""
    from .resnet_workload import approx_qparams, load_float_weights
    if seed is not None:
        torch.manual_seed(seed)
    fp = ViTForImageClassification(image_size, patch_size, 3, hidden, layers, heads, mlp, num_labels)
    if weights:
        load_float_weights(fp, weights)
    assert hidden % heads == 0 and image_size % patch_size == 0
    return QuantizedVisionTransformerForImageClassification(fp, input_size=(1, 3, image_size, image_size),
                                                            flatten_token_rows=flatten_token_rows,
                                                            **approx_qparams(**cfg))


def vit_approx_macs_per_image(image_size=224, patch_size=16, hidden=768, layers=12, mlp=3072, num_labels=1000):
    """Approx-MACs of one image: per layer Q, K, V, attention output (T x D x D each) and the
    MLP (2 x T x D x mlp), plus the classifier on the class token; T = patches + 1."""
    T = (image_size // patch_size) ** 2 + 1
    return layers * (4 * T * hidden * hidden + 2 * T * hidden * mlp) + hidden * num_labels


__all__ = ["ViTForImageClassification", "QuantizedVisionTransformerForImageClassification", "vit_b16_approx",
           "vit_approx_macs_per_image"]
