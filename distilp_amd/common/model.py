"""Model profile schemas (solver scalar form and profiler per-layer form).

Field names / defaults follow `src/distilp/common/model.py:12-251` of the
reference. `ModelProfileSplit.to_model_profile` reproduces the reference's
reduction (model.py:193-251): layer index 1 is the "typical layer", f_q and
f_out come from the requested phase, Q = quantization.
"""

from __future__ import annotations

from typing import Dict, List, Literal, Optional

from pydantic import BaseModel, Field

from .types import ModelPhase, QuantizationLevel


class ModelProfile(BaseModel):
    """Scalar model description consumed by the HALDA solver."""

    # architecture
    L: int = 0
    hk: int = 0
    ek: int = 0
    hv: int = 0
    ev: int = 0
    n_kv: int = 0
    e_embed: int = 0
    V: int = 0

    # solver scalars: typical-layer bytes / FLOPs
    b_layer: int = 0
    b_in: int = 0
    b_out: int = 0
    f_q: Dict[str, float] = Field(default_factory=dict)  # "b_1" -> FLOPs
    f_out: Dict[str, float] = Field(default_factory=dict)
    Q: QuantizationLevel = "F16"

    # optional per-layer arrays (profiler form)
    b_layers: Optional[List[int]] = None
    b_i_layers: Optional[List[int]] = None
    b_o_layers: Optional[List[int]] = None
    f_q_layers: Optional[Dict[str, List[float]]] = None

    seq_len: int = 0
    quantization: QuantizationLevel = "F16"

    # MoE description (not used by the dense HALDA formulation)
    is_moe: bool = False
    n_routed_experts: int = 0
    n_shared_experts: int = 0
    experts_per_token: int = 0
    moe_intermediate_size: int = 0
    moe_layer_freq: int = 1
    first_k_dense_replace: int = 0
    total_moe_layers: int = 0
    moe_layer_indices: Optional[List[int]] = None

    attn_bytes: Optional[List[int]] = None
    attn_flops: Optional[Dict[str, List[float]]] = None
    bytes_per_expert: Optional[Dict[int, int]] = None
    bytes_shared_experts: Optional[Dict[int, int]] = None
    flops_per_expert: Optional[Dict[int, float]] = None
    flops_shared_experts: Optional[Dict[int, float]] = None
    router_flops: Optional[Dict[int, float]] = None
    router_bytes: Optional[Dict[int, int]] = None
    flops_per_active_expert_per_token: Optional[Dict[int, float]] = None

    def print_summary(self) -> None:
        mib = 1024**2
        bar = "=" * 60
        print(f"\n{bar}\nModel Profile:\n{bar}")
        print(f"  Layers (L): {self.L}")
        if self.b_layer > 0:
            print(f"  Bytes per layer: {self.b_layer / mib:.1f} MB")
        if self.b_in > 0:
            print(f"  Input bytes: {self.b_in / mib:.1f} MB")
        if self.b_out > 0:
            print(f"  Output bytes: {self.b_out / mib:.1f} MB")
        print(f"  Attention heads (k/v): {self.hk}/{self.hv}")
        print(f"  Head dimensions (k/v): {self.ek}/{self.ev}")
        print(f"  KV cache tokens: {self.n_kv}")
        print(f"  Embedding dimension: {self.e_embed}")
        print(f"  Vocabulary size: {self.V}")
        print(f"  Quantization: {self.Q}")


class ModelProfilePhased(BaseModel):
    """Prefill/decode pair (reference model.py:107-133)."""

    prefill: ModelProfile
    decode: ModelProfile

    def to_model_profile(self, phase: Literal["decode", "prefill"] = "decode") -> ModelProfile:
        if phase not in ("decode", "prefill"):
            raise ValueError(f"Invalid phase: {phase}. Must be 'decode' or 'prefill'.")
        return self.decode if phase == "decode" else self.prefill


class ModelProfileSplit(BaseModel):
    """Profiler output: per-layer arrays (index 0 = embedding) split by phase."""

    b: List[int]
    b_i: List[int]
    b_o: List[int]
    L: int
    hk: int
    hv: int
    ek: int
    ev: int
    n_kv: int
    e_embed: int
    V: int
    seq_len: int
    f_q: Dict[ModelPhase, Dict[str, List[float]]]
    f_out: Dict[ModelPhase, Dict[str, float]]
    quantization: QuantizationLevel

    is_moe: bool = False
    n_routed_experts: int = 0
    n_shared_experts: int = 0
    experts_per_token: int = 0
    moe_intermediate_size: int = 0
    moe_layer_freq: int = 0
    first_k_dense_replace: int = 0
    total_moe_layers: int = 0
    moe_layer_indices: List[int] = Field(default_factory=list)

    attn_bytes: List[int] = Field(default_factory=list)
    attn_flops: Dict[ModelPhase, Dict[str, List[float]]] = Field(default_factory=dict)
    bytes_per_expert: Dict[int, int] = Field(default_factory=dict)
    bytes_shared_experts: Dict[int, int] = Field(default_factory=dict)
    flops_per_expert: Dict[int, float] = Field(default_factory=dict)
    flops_shared_experts: Dict[int, float] = Field(default_factory=dict)
    router_flops: Dict[int, float] = Field(default_factory=dict)
    router_bytes: Dict[int, int] = Field(default_factory=dict)
    flops_per_active_expert_per_token: Dict[int, float] = Field(default_factory=dict)

    def to_model_profile(self, phase: Literal["decode", "prefill"] = "decode") -> ModelProfile:
        """Collapse to the solver's scalar form using layer 1 as the typical layer."""

        def layer1(arr: List[int]) -> int:
            return arr[1] if len(arr) > 1 else 0

        per_batch = self.f_q[phase]
        f_q = {key: vals[1] for key, vals in per_batch.items() if isinstance(vals, list) and len(vals) > 1}
        return ModelProfile(
            L=self.L,
            b_layer=layer1(self.b),
            b_in=layer1(self.b_i),
            b_out=layer1(self.b_o),
            hk=self.hk,
            ek=self.ek,
            hv=self.hv,
            ev=self.ev,
            n_kv=self.n_kv,
            e_embed=self.e_embed,
            V=self.V,
            f_q=f_q,
            f_out=self.f_out[phase],
            Q=self.quantization,
            quantization=self.quantization,
            is_moe=self.is_moe,
            n_routed_experts=self.n_routed_experts,
            n_shared_experts=self.n_shared_experts,
            experts_per_token=self.experts_per_token,
            moe_intermediate_size=self.moe_intermediate_size,
            moe_layer_freq=self.moe_layer_freq,
            first_k_dense_replace=self.first_k_dense_replace,
            total_moe_layers=self.total_moe_layers,
            moe_layer_indices=self.moe_layer_indices,
            attn_bytes=self.attn_bytes,
            attn_flops=self.attn_flops.get(phase, {}),
            bytes_per_expert=self.bytes_per_expert,
            bytes_shared_experts=self.bytes_shared_experts,
            flops_per_expert=self.flops_per_expert,
            flops_shared_experts=self.flops_shared_experts,
            router_flops=self.router_flops,
            router_bytes=self.router_bytes,
            flops_per_active_expert_per_token=self.flops_per_active_expert_per_token,
        )
