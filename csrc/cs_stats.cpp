// Statistics of the chunkserver's native components as JSON objects, one key list per
// component: the Python bindings turn them into dicts and dfs_chunkserver serves them on
// /stats, so both processes report the same names (bench.py and the tests read them).
#include "cs_stats.h"

#include "chunk_store.h"
#include "cs_agent.h"
#include "cs_grpc.h"
#include "fastpath.h"
#include "replication.h"

#include <utility>

namespace dfs {

Json stats_json(const StoreStats& t) {
  Json d = Json::object();
  d.set("blocks", t.blocks);
  d.set("bytes", t.bytes);
  d.set("hbm_capacity", t.hbm_capacity);
  d.set("hbm_used", t.hbm_used);
  d.set("hbm_resident_blocks", t.hbm_resident_blocks);
  d.set("dirty_blocks", t.dirty_blocks);
  d.set("spill_queue", t.spill_queue);
  d.set("evictions", t.evictions);
  d.set("promotions", t.promotions);
  d.set("mirror_hits", t.mirror_hits);
  d.set("mirror_bytes", t.mirror_bytes);
  d.set("io_threads_spawned", t.io_threads_spawned);
  d.set("final_name_writes", t.final_name_writes);
  d.set("direct_writes", t.direct_writes);
  d.set("crc_mismatches", t.crc_mismatches);
  d.set("scrub_transient", t.scrub_transient);
  d.set("gpu_kernel_launches", t.gpu_kernel_launches);
  d.set("disk_gate_waits", t.disk_gate_waits);
  d.set("direct_dma", t.direct_dma);
  d.set("fused_reads", t.fused_reads);
  d.set("fused_writes", t.fused_writes);
  d.set("pulled_recvs", t.pulled_recvs);
  d.set("pulled_host_appends", t.pulled_host_appends);
  d.set("sliced_stages", t.sliced_stages);
  d.set("staged_dma", t.staged_dma);
  d.set("host_registered_bytes", t.host_registered_bytes);
  d.set("journal", t.journal);
  d.set("journal_records", t.journal_records);
  d.set("journal_bytes", t.journal_bytes);
  d.set("journal_commits", t.journal_commits);
  d.set("journal_sync_rounds", t.journal_sync_rounds);
  d.set("journal_mode", t.journal_mode);
  d.set("journal_tombstones", t.journal_tombstones);
  d.set("journal_supersedes", t.journal_supersedes);
  d.set("journal_segs_in_use", t.journal_segs_in_use);
  d.set("journal_segs_marked", t.journal_segs_marked);
  d.set("journal_replay_verified", t.journal_replay_verified);
  d.set("journal_live_records", t.journal_live_records);
  d.set("journal_live_bytes", t.journal_live_bytes);
  d.set("journal_used_bytes", t.journal_used_bytes);
  d.set("journal_grow_blocked", t.journal_grow_blocked);
  d.set("relocated_blocks", t.relocated_blocks);
  d.set("relocated_bytes", t.relocated_bytes);
  d.set("compactions", t.compactions);
  d.set("export_deferred_headroom", t.export_deferred_headroom);
  d.set("scrub_device_blocks", t.scrub_device_blocks);
  d.set("lane_waits", t.lane_waits);
  d.set("lane_wait_ns", t.lane_wait_ns);
  d.set("journal_full_waits", t.journal_full_waits);
  d.set("journal_segs", t.journal_segs);
  d.set("journal_segs_free", t.journal_segs_free);
  d.set("journal_segs_retired", t.journal_segs_retired);
  d.set("journal_replayed", t.journal_replayed);
  d.set("journal_replay_skipped", t.journal_replay_skipped);
  d.set("journal_failed", t.journal_failed);
  d.set("materialized_blocks", t.materialized_blocks);
  d.set("materialized_bytes", t.materialized_bytes);
  d.set("materialize_pending", t.materialize_pending);
  d.set("materialize_batches", t.materialize_batches);
  d.set("materialize_errors", t.materialize_errors);
  d.set("materialize_last_error", t.materialize_last_error);
  d.set("journal_prepare_errors", t.journal_prepare_errors);
  d.set("journal_segs_filled", t.journal_segs_filled);
  d.set("journal_fill_bytes", t.journal_fill_bytes);
  d.set("journal_parts_unready", t.journal_parts_unready);
  d.set("journal_spares_missing", t.journal_spares_missing);
  d.set("journal_grow_deferred", t.journal_grow_deferred);
  d.set("journal_mark_preflushes", t.journal_mark_preflushes);
  d.set("journal_reserve_markers", t.journal_reserve_markers);
  d.set("delete_tomb_failures", t.delete_tomb_failures);
  d.set("export_busy_polls", t.export_busy_polls);
  d.set("journal_sync_ns", t.journal_sync_ns);
  d.set("journal_bypassed", t.journal_bypassed);
  d.set("journal_commit_ns", t.journal_commit_ns);
  d.set("journal_last_error", t.journal_last_error);
  return d;
}

Json stats_json(const CsAgentStats& t) {
  Json d = Json::object();
  d.set("agent_heartbeats", t.heartbeats);
  d.set("agent_heartbeat_failures", t.heartbeat_failures);
  d.set("agent_commands", t.commands);
  d.set("agent_map_refreshes", t.map_refreshes);
  d.set("agent_replicate_engine", t.replicate_engine);
  d.set("agent_replicate_grpc", t.replicate_grpc);
  d.set("agent_replicate_failed", t.replicate_failed);
  d.set("agent_reconstructs", t.reconstructs);
  d.set("agent_reconstruct_device", t.reconstruct_device);
  d.set("agent_reconstruct_failed", t.reconstruct_failed);
  d.set("agent_encodes", t.encodes);
  d.set("agent_encode_failed", t.encode_failed);
  d.set("agent_recoveries", t.recoveries);
  d.set("agent_recovery_failed", t.recovery_failed);
  d.set("agent_deletes", t.deletes);
  d.set("agent_moves", t.moves);
  d.set("agent_scrubs", t.scrubs);
  d.set("agent_scrub_bad", t.scrub_bad);
  d.set("agent_ec_gpu", t.ec_gpu);
  d.set("agent_ec_cpu", t.ec_cpu);
  return d;
}

Json stats_json(const FpStats& t) {
  Json d = Json::object();
  d.set("fp_writes", t.writes);
  d.set("fp_reads", t.reads);
  d.set("fp_fenced", t.fenced);
  d.set("fp_punts", t.punts);
  d.set("fp_connections", t.connections);
  d.set("fp_replicas_in", t.replicas_in);
  d.set("fp_rccl_forwards", t.rccl_forwards);
  d.set("fp_shm_forwards", t.shm_forwards);
  d.set("fp_forward_failures", t.forward_failures);
  d.set("fp_replica_failures", t.replica_failures);
  d.set("fp_p2p_fallbacks", t.p2p_fallbacks);
  d.set("fp_rejected_peers", t.rejected_peers);
  d.set("fp_ec_ops", t.ec_ops);
  d.set("fp_heals_out", t.heals_out);
  d.set("fp_heals_in", t.heals_in);
  d.set("fp_sliced_writes", t.sliced_writes);
  d.set("fp_ec_device_writes", t.ec_device_writes);
  d.set("fp_ec_shard_forwards", t.ec_shard_forwards);
  d.set("fp_ec_device_reads", t.ec_device_reads);
  d.set("fp_ec_device_decodes", t.ec_device_decodes);
  d.set("fp_ec_gathered", t.ec_gathered);
  d.set("fp_ec_device_fallbacks", t.ec_device_fallbacks);
  d.set("fp_chain_writes", t.chain_writes);
  d.set("fp_chain_stage_ns", t.chain_stage_ns);
  d.set("fp_chain_forward_ns", t.chain_forward_ns);
  d.set("fp_desc_calls", t.desc_calls);
  d.set("fp_desc_ns", t.desc_ns);
  return d;
}

Json stats_json(const ReplStats& t) {
  Json d = Json::object();
  d.set("bytes_sent", t.bytes_sent);
  d.set("bytes_recv", t.bytes_recv);
  d.set("blocks_sent", t.blocks_sent);
  d.set("blocks_recv", t.blocks_recv);
  d.set("pair_failures", t.pair_failures);
  d.set("pair_opens", t.pair_opens);
  d.set("open_attempts", t.open_attempts);
  d.set("turn_timeouts", t.turn_timeouts);
  d.set("stale_generation", t.stale_generation);
  d.set("channel_waits", t.channel_waits);
  d.set("parked_extents", t.parked_extents);
  d.set("reaped_extents", t.reaped_extents);
  for (auto [k, v] : {std::pair<const char*, uint64_t>{"send_calls", t.send_calls}, {"send_stage_ns", t.send_stage_ns},
                      {"send_turn_ns", t.send_turn_ns}, {"send_post_ns", t.send_post_ns}, {"wait_send_ns", t.wait_send_ns},
                      {"recv_calls", t.recv_calls}, {"recv_turn_ns", t.recv_turn_ns}, {"recv_land_ns", t.recv_land_ns},
                      {"recv_finish_ns", t.recv_finish_ns}})
    d.set(k, v);
  for (auto& kv : t.sent_to) d.set("link_sent_to_" + std::to_string(kv.first), kv.second);
  for (auto& kv : t.recv_from) d.set("link_recv_from_" + std::to_string(kv.first), kv.second);
  return d;
}

Json stats_json(const CsGrpcStats& t, uint64_t calls) {
  Json d = Json::object();
  d.set("native_grpc_calls", calls);
  d.set("native_grpc_writes", t.native_writes);
  d.set("native_grpc_reads", t.native_reads);
  d.set("native_grpc_replicates", t.native_replicates);
  d.set("native_grpc_fallbacks", t.fallbacks);
  d.set("native_grpc_forwards", t.grpc_forwards);
  d.set("native_grpc_forward_failures", t.grpc_forward_failures);
  d.set("native_grpc_recoveries", t.recoveries);
  d.set("native_grpc_shm_writes", t.shm_writes);
  d.set("native_grpc_shm_reads", t.shm_reads);
  return d;
}

void merge_into(Json* dst, const Json& src, const std::string& prefix) {
  for (const auto& kv : src.fields()) dst->set(prefix + kv.first, kv.second);
}

}  // namespace dfs
