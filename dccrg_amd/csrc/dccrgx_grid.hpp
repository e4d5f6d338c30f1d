// Host driver functions shared by grid.hip (halo, refinement, migration,
// sweeps) and api.hip (the C ABI).
#pragma once

#include "dccrgx_internal.hpp"

namespace dccrgx {

std::vector<Field*> transfer_fields(Grid& g);
Field& field(Grid& g, int fid);
Field& fixed_field(Grid& g, int fid);  // EINVAL for a variable-size field
std::vector<Field*> var_transfer_fields(Grid& g);
void ensure_scratch(Grid& g, Field& f);
void commit(Grid& g, Field& f);
void region_range(const Grid& g, int region, size_t& s0, size_t& s1);
void drain_timing(Grid& g);

void halo_start(Grid& g);
void halo_wait(Grid& g);
UserHood& ensure_uhood(Grid& g, int id);
HaloPlan& plan_of(Grid& g, int hood);
void uhood_halo(Grid& g, int id);
size_t halo_pack_peer(Grid& g, int hood, int peer, uint8_t* buf, size_t cap);
void halo_place_peer(Grid& g, int hood, int peer, const uint8_t* buf, size_t bytes);
void halo_message_size(Grid& g, int hood, int peer, size_t& sb, size_t& rb);

void stop_refining_impl(Grid& g);  // the created cells in Grid::new_cells

void initialize_balance_load_impl(Grid& g, bool use_partitioner, const uint64_t* cells, const int32_t* procs,
                                  size_t n);
// partition.hip: recursive coordinate bisection of the leaves (the new
// owner of every local cell, cells ascending); collective
void rcb_partition(Grid& g, std::vector<uint64_t>& cells, std::vector<int32_t>& owners);
void continue_balance_load_impl(Grid& g);
void finish_balance_load_impl(Grid& g);
void migration_message_size(Grid& g, int peer, size_t& sb, size_t& rb);
void migration_pack_peer(Grid& g, int peer, uint8_t* buf, size_t cap);
void migration_place_peer(Grid& g, int peer, const uint8_t* buf, size_t bytes);

std::vector<uint64_t> cells_by_criteria(Grid& g, const int32_t* crit, size_t nc, bool exact, int hood);
int64_t host_slot_of(Grid& g, uint64_t id);
bool gol_slab_plan(Grid& g, std::vector<GolBox>& inner, std::vector<GolBox>& outer);

}  // namespace dccrgx
