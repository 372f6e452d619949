"""turtle_kv_amd -- MI355X-native AMQ filter engine for TurtleKV's per-leaf Bloom / VQF
build-and-probe path.  Compute runs in HIP kernels (libtkv_amq.so); this
package is the host-side mirror of the reference's filter API."""
from . import abi
from .abi import BLOOM, VQF, TkvAmqError
from .filters import (BoolStatus, FilterPage, FilterPlan, KeyBatch, KeyQuery, PackedVqfFilter,
                      build_all_filters, build_bloom_filter_for_leaf, build_filter_for_leaf_in_job,
                      build_quotient_filter_for_leaf, filter_bits_per_key, gen_keys16,
                      bloom_query_hashes, bloom_probe_hashed, HostFilterPipeline,
                      plan_filters, probe_filters, vqf_filter_load_factor, vqf_hash_val,
                      vqf_nslots_for_size, vqf_probe_hashed, vqf_required_size, key_views,
                      stage_keys, BloomFilterMetrics, QuotientFilterMetrics,
                      plan_filter_stats, record_filter_metrics, TreeOptions, plan_filter_pages,
                      page_header_fields, ProbeMetrics, KeyQueryMetrics)

__all__ = [
    "abi", "BLOOM", "VQF", "TkvAmqError", "BoolStatus", "FilterPage", "FilterPlan", "KeyBatch",
    "KeyQuery", "PackedVqfFilter", "build_all_filters", "build_bloom_filter_for_leaf",
    "build_filter_for_leaf_in_job", "build_quotient_filter_for_leaf", "filter_bits_per_key",
    "gen_keys16", "plan_filters", "probe_filters", "vqf_filter_load_factor", "vqf_hash_val",
    "vqf_nslots_for_size", "vqf_probe_hashed", "vqf_required_size", "bloom_query_hashes",
    "bloom_probe_hashed", "HostFilterPipeline", "key_views", "stage_keys",
    "BloomFilterMetrics", "QuotientFilterMetrics", "plan_filter_stats", "record_filter_metrics",
    "TreeOptions", "plan_filter_pages", "page_header_fields", "ProbeMetrics", "KeyQueryMetrics",
]
