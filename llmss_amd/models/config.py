"""Architecture description shared by every model family.

The reference builds each family from a ``transformers.PretrainedConfig`` subclass and
``PreTrainedModel`` glue (``gptj_modeling.py:320-354``, ``gpt_bigcode_modeling.py:417-462``).
Here a single flat dataclass captures everything the native decoder needs; it is parsed
from a HF ``config.json`` (no ``transformers`` import on the hot path) or built from a named
preset for synthetic/random-init runs (bench, smoke tests).

Families (``MODEL_REGISTRY`` keys, reference ``custom_modeling/__init__.py:4-7`` had only
``gptj`` and ``gpt_bigcode``):

* ``gpt2``        - LayerNorm, learned positions, Conv1D fused c_attn, GELU-tanh, tied head.
* ``gptj``        - LayerNorm, *parallel* residual block, interleaved partial RoPE,
                    separate q/k/v without bias, lm_head with bias (``gptj_modeling.py``).
* ``gpt_bigcode`` - LayerNorm, learned positions, MQA (or MHA) fused c_attn, tied head
                    (``gpt_bigcode_modeling.py``).
* ``llama``       - RMSNorm, half-rotate RoPE, GQA, SwiGLU, untied head.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass, field, replace
from typing import Any, Dict, Optional


@dataclass
class ModelConfig:
    model_type: str
    vocab_size: int
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    max_position_embeddings: int
    norm: str = "layernorm"  # "layernorm" | "rmsnorm"
    norm_eps: float = 1e-5
    activation: str = "gelu_tanh"  # "gelu_tanh" | "gelu" | "silu_glu" | "relu"
    position: str = "learned"  # "learned" | "rope"
    rope_style: str = "neox"  # "neox" (half rotate) | "gptj" (interleaved pairs)
    rotary_dim: int = 0
    rope_theta: float = 10000.0
    parallel_block: bool = False  # GPT-J: attn and mlp read the same LN output
    tie_word_embeddings: bool = False
    qkv_bias: bool = False
    out_bias: bool = False
    mlp_bias: bool = False
    lm_head_bias: bool = False
    conv1d_weights: bool = False  # GPT-2 stores [in, out] Conv1D weights
    fused_qkv_name: Optional[str] = None  # checkpoint tensor name of the fused c_attn, if any
    bos_token_id: Optional[int] = None
    eos_token_id: Optional[int] = None
    pad_token_id: Optional[int] = None
    extra: Dict[str, Any] = field(default_factory=dict)

    # ---------------------------------------------------------------- derived
    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def gated_mlp(self) -> bool:
        return self.activation == "silu_glu"

    @property
    def n_positions(self) -> int:  # reference name (generate.py:60)
        return self.max_position_embeddings

    def num_params(self) -> int:
        h, f, v = self.hidden_size, self.intermediate_size, self.vocab_size
        attn = h * (self.q_size + 2 * self.kv_size) + self.q_size * h
        mlp = (3 if self.gated_mlp else 2) * h * f
        per_layer = attn + mlp + 4 * h
        emb = v * h + (self.max_position_embeddings * h if self.position == "learned" else 0)
        head = 0 if self.tie_word_embeddings else v * h
        return self.num_layers * per_layer + emb + head

    def to_dict(self) -> Dict[str, Any]:
        return asdict(self)

    # ---------------------------------------------------------------- parsing
    @classmethod
    def from_hf_dict(cls, d: Dict[str, Any]) -> "ModelConfig":
        mt = d.get("model_type")
        common = dict(
            bos_token_id=d.get("bos_token_id"),
            eos_token_id=_first(d.get("eos_token_id")),
            pad_token_id=d.get("pad_token_id"),
        )
        if mt == "gpt2":
            h, nh = d["n_embd"], d["n_head"]
            return cls(
                model_type="gpt2", vocab_size=d["vocab_size"], hidden_size=h, num_layers=d["n_layer"],
                num_heads=nh, num_kv_heads=nh, head_dim=h // nh,
                intermediate_size=d.get("n_inner") or 4 * h, max_position_embeddings=d["n_positions"],
                norm="layernorm", norm_eps=d.get("layer_norm_epsilon", 1e-5),
                activation=_act(d.get("activation_function", "gelu_new")), position="learned",
                tie_word_embeddings=d.get("tie_word_embeddings", True), qkv_bias=True, out_bias=True,
                mlp_bias=True, conv1d_weights=True, fused_qkv_name="c_attn", **common,
            )
        if mt == "gptj":
            h, nh = d["n_embd"], d["n_head"]
            hd = h // nh
            return cls(
                model_type="gptj", vocab_size=d["vocab_size"], hidden_size=h, num_layers=d["n_layer"],
                num_heads=nh, num_kv_heads=nh, head_dim=hd,
                intermediate_size=d.get("n_inner") or 4 * h, max_position_embeddings=d["n_positions"],
                norm="layernorm", norm_eps=d.get("layer_norm_epsilon", 1e-5),
                activation=_act(d.get("activation_function", "gelu_new")), position="rope",
                rope_style="gptj", rotary_dim=d.get("rotary_dim") or hd, parallel_block=True,
                tie_word_embeddings=d.get("tie_word_embeddings", False), qkv_bias=False, out_bias=False,
                mlp_bias=True, lm_head_bias=True, **common,
            )
        if mt == "gpt_bigcode":
            h, nh = d["n_embd"], d["n_head"]
            mq = d.get("multi_query", True)
            return cls(
                model_type="gpt_bigcode", vocab_size=d["vocab_size"], hidden_size=h, num_layers=d["n_layer"],
                num_heads=nh, num_kv_heads=1 if mq else nh, head_dim=h // nh,
                intermediate_size=d.get("n_inner") or 4 * h, max_position_embeddings=d["n_positions"],
                norm="layernorm", norm_eps=d.get("layer_norm_epsilon", 1e-5),
                activation=_act(d.get("activation_function", "gelu_pytorch_tanh")), position="learned",
                tie_word_embeddings=d.get("tie_word_embeddings", True), qkv_bias=True, out_bias=True,
                mlp_bias=True, fused_qkv_name="c_attn", **common,
            )
        if mt in ("llama", "mistral"):
            h, nh = d["hidden_size"], d["num_attention_heads"]
            hd = d.get("head_dim") or h // nh
            return cls(
                model_type="llama", vocab_size=d["vocab_size"], hidden_size=h, num_layers=d["num_hidden_layers"],
                num_heads=nh, num_kv_heads=d.get("num_key_value_heads") or nh, head_dim=hd,
                intermediate_size=d["intermediate_size"],
                max_position_embeddings=d.get("max_position_embeddings", 4096),
                norm="rmsnorm", norm_eps=d.get("rms_norm_eps", 1e-6), activation="silu_glu", position="rope",
                rope_style="neox", rotary_dim=hd, rope_theta=_rope_theta(d),
                tie_word_embeddings=d.get("tie_word_embeddings", False),
                qkv_bias=d.get("attention_bias", False), out_bias=d.get("attention_bias", False),
                mlp_bias=d.get("mlp_bias", False), **common,
            )
        raise ValueError(f"unsupported model_type {mt!r}; supported: gpt2, gptj, gpt_bigcode, llama")

    @classmethod
    def from_pretrained(cls, path: str) -> "ModelConfig":
        with open(os.path.join(path, "config.json")) as f:
            return cls.from_hf_dict(json.load(f))


def _first(x):
    if isinstance(x, (list, tuple)):
        return x[0] if x else None
    return x


def _act(name: str) -> str:
    name = name.lower()
    if name in ("gelu_new", "gelu_pytorch_tanh", "gelu_fast", "gelu_tanh"):
        return "gelu_tanh"
    if name in ("gelu",):
        return "gelu"
    if name in ("relu",):
        return "relu"
    if name in ("silu", "swish"):
        return "silu_glu"
    raise ValueError(f"unsupported activation {name}")


def _rope_theta(d: Dict[str, Any]) -> float:
    if "rope_theta" in d:
        return float(d["rope_theta"])
    rp = d.get("rope_parameters") or {}
    return float(rp.get("rope_theta", 10000.0))


# -------------------------------------------------------------------- presets
# Public HF architectures used for random-init benches and smoke tests.
_PRESETS: Dict[str, Dict[str, Any]] = {
    "gpt2": dict(model_type="gpt2", n_embd=768, n_layer=12, n_head=12, n_positions=1024, vocab_size=50257),
    "gpt2-medium": dict(model_type="gpt2", n_embd=1024, n_layer=24, n_head=16, n_positions=1024, vocab_size=50257),
    "gpt2-xl": dict(model_type="gpt2", n_embd=1600, n_layer=48, n_head=25, n_positions=1024, vocab_size=50257),
    "gptj-6b": dict(model_type="gptj", n_embd=4096, n_layer=28, n_head=16, n_positions=2048, vocab_size=50400,
                    rotary_dim=64),
    "kogpt-j-350m": dict(model_type="gptj", n_embd=1024, n_layer=20, n_head=16, n_positions=2048,
                         vocab_size=51200, rotary_dim=64),
    "santacoder": dict(model_type="gpt_bigcode", n_embd=2048, n_layer=24, n_head=16, n_positions=2048,
                       vocab_size=49280, multi_query=True),
    "starcoder": dict(model_type="gpt_bigcode", n_embd=6144, n_layer=40, n_head=48, n_positions=8192,
                      vocab_size=49152, multi_query=True),
    "llama2-7b": dict(model_type="llama", hidden_size=4096, num_hidden_layers=32, num_attention_heads=32,
                      num_key_value_heads=32, intermediate_size=11008, vocab_size=32000,
                      max_position_embeddings=4096),
    "llama2-13b": dict(model_type="llama", hidden_size=5120, num_hidden_layers=40, num_attention_heads=40,
                       num_key_value_heads=40, intermediate_size=13824, vocab_size=32000,
                       max_position_embeddings=4096),
    "llama2-70b": dict(model_type="llama", hidden_size=8192, num_hidden_layers=80, num_attention_heads=64,
                       num_key_value_heads=8, intermediate_size=28672, vocab_size=32000,
                       max_position_embeddings=4096),
    # tiny shapes for tests
    "tiny-gpt2": dict(model_type="gpt2", n_embd=64, n_layer=2, n_head=4, n_positions=128, vocab_size=211),
    "tiny-gptj": dict(model_type="gptj", n_embd=64, n_layer=2, n_head=4, n_positions=128, vocab_size=211,
                      rotary_dim=8),
    "tiny-bigcode": dict(model_type="gpt_bigcode", n_embd=64, n_layer=2, n_head=4, n_positions=128,
                         vocab_size=211, multi_query=True),
    "tiny-llama": dict(model_type="llama", hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                       num_key_value_heads=2, intermediate_size=160, vocab_size=211,
                       max_position_embeddings=128),
    # TP up to 8 (16 q / kv heads: 2 per rank at TP=8, as Llama-2-7B's 32 give 4)
    "tiny-llama16h": dict(model_type="llama", hidden_size=256, num_hidden_layers=2, num_attention_heads=16,
                          num_key_value_heads=16, intermediate_size=512, vocab_size=211,
                          max_position_embeddings=128),
}


def preset_names():
    return sorted(_PRESETS)


def preset_hf_dict(name: str) -> Dict[str, Any]:
    if name not in _PRESETS:
        raise KeyError(f"unknown preset {name!r}; known: {preset_names()}")
    return dict(_PRESETS[name])


def get_preset(name: str, **overrides) -> ModelConfig:
    cfg = ModelConfig.from_hf_dict(preset_hf_dict(name))
    return replace(cfg, **overrides) if overrides else cfg
