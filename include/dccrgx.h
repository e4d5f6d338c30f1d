/*
 * dccrgx — C ABI of the MI355X-native dccrg neighbor-stencil + halo path.
 *
 * One opaque grid per process (one process per GPU).  Cell payloads live in
 * HBM as structure-of-arrays "fields"; every field is indexed by a *slot*:
 *
 *     [0, n_inner)              local cells without remote neighbors
 *     [n_inner, n_local)        local cells with remote neighbors
 *                               (both runs in ascending id on unrefined grids,
 *                               in Morton order of the cells' min corners when
 *                               max refinement level > 0, for locality)
 *     [n_local, n_local+n_recv) copies of remote neighbors, grouped by owner
 *                               (ascending rank), ascending id inside a group
 *                               = the halo exchange wire order
 *     [.., n_slots)             remote cells that only have local cells as
 *                               neighbors_to (no payload is ever received)
 *
 * State per rank is the rank's own leaves plus the "ghost" leaves around
 * them (within max(neighborhood length, 1) level-0 cells), never the whole
 * grid: the reference's global cell_process map (dccrg.hpp:7197) has no
 * counterpart.
 *
 * Every entry point returns 0 on success and a negative code on failure;
 * dccrgx_last_error() then describes the failure.  Every function cites the
 * reference interface (lkotipal/dccrg @ 2024-10-24, dccrg.hpp unless noted)
 * it replaces.
 */
#ifndef DCCRGX_H
#define DCCRGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dccrgx_grid dccrgx_grid;

#define DCCRGX_ABI_VERSION 10 /* dccrgx_abi_version() of a matching library */

#define DCCRGX_OK 0
#define DCCRGX_EINVAL -1   /* bad argument / wrong state  (std::invalid_argument) */
#define DCCRGX_EHIP -2     /* HIP runtime failure */
#define DCCRGX_ECOMM -3    /* RCCL failure */
#define DCCRGX_ERANGE -4   /* caller buffer too small; *n holds the needed size */
#define DCCRGX_ENOTFOUND -5 /* unknown cell (reference returns nullptr) */

/* cell selections for dccrgx_get_cells (iterator ranges dccrg.hpp:7478-7602) */
#define DCCRGX_CELLS_LOCAL 0   /* local_cells()  */
#define DCCRGX_CELLS_INNER 1   /* inner_cells()  */
#define DCCRGX_CELLS_OUTER 2   /* outer_cells()  */
#define DCCRGX_CELLS_REMOTE 3  /* remote_cells() = remote_cells_on_process_boundary */
#define DCCRGX_CELLS_ALL 4     /* all_cells()    */

/* sweep regions */
#define DCCRGX_REGION_ALL 0
#define DCCRGX_REGION_INNER 1
#define DCCRGX_REGION_OUTER 2

const char* dccrgx_last_error(void);
int dccrgx_abi_version(void);

/* ---- communicator / lifetime ---------------------------------------------
 * dccrgx_get_unique_id: rank 0 creates the 128-byte RCCL bootstrap id that the
 * caller broadcasts (replaces Dccrg::initialize(MPI_Comm) 472-552's
 * MPI_Comm_dup, 7622-7687).  nccl_id may be NULL when size == 1. */
int dccrgx_get_unique_id(void* out_128_bytes);
int dccrgx_create(int rank, int size, int device, const void* nccl_id, dccrgx_grid** out);
int dccrgx_destroy(dccrgx_grid* g);

/* A host transport instead of RCCL (ranks sharing one GPU, MPI programs,
 * tests): one grouped point-to-point exchange with every rank - send
 * send_bytes[p] bytes from send[p] to rank p and receive recv_bytes[p] bytes
 * from rank p into recv[p] (entries of 0 bytes and the own rank post
 * nothing; all buffers are host memory).  Every rank calls it the same number
 * of times in the same order, as MPI point-to-point calls in the reference
 * (start_user_data_transfers 10564-10997).  Returns 0 on success.  The
 * library builds its collectives (All_Gather, Allreduce) and the halo and
 * migration payload transfers on it. */
typedef int (*dccrgx_exchange_fn)(void* ctx, const void* const* send, const size_t* send_bytes, void* const* recv,
                                  const size_t* recv_bytes);
int dccrgx_create_with_exchange(int rank, int size, int device, dccrgx_exchange_fn fn, void* ctx, dccrgx_grid** out);
/* number of visible GPUs (for choosing a device per rank) */
int dccrgx_device_count(int* n);

/* ---- setup, before initialize (dccrg.hpp:8120-8230) ---------------------- */
int dccrgx_set_initial_length(dccrgx_grid* g, const uint64_t length[3]);   /* 8120 */
int dccrgx_set_maximum_refinement_level(dccrgx_grid* g, int level);        /* 8154 */
int dccrgx_set_periodic(dccrgx_grid* g, int x, int y, int z);              /* 8183 */
int dccrgx_set_neighborhood_length(dccrgx_grid* g, unsigned length);       /* 8206 */
int dccrgx_get_maximum_refinement_level(dccrgx_grid* g, int* level);
/* the setup as the library holds it, e.g. after load_grid_data read it from
 * a file: length in level-0 cells, periodicity (ABI 8) */
int dccrgx_get_initial_length(dccrgx_grid* g, uint64_t length[3]);
int dccrgx_get_periodic(dccrgx_grid* g, int periodic[3]);
/* get_neighborhood_length (6725): the length set, or read from a grid file
 * by load_grid_data (ABI 8) */
int dccrgx_get_neighborhood_length(dccrgx_grid* g, unsigned* length);
/* initialize(): level-0 cells, block partition (create_level_0_cells
 * 7967-8102), device neighbor build (initialize_neighbors 8240-8289 and
 * update_remote_neighbor_info / send-receive lists 8590-9309).  472 */
int dccrgx_initialize(dccrgx_grid* g);
/* Cartesian_Geometry::set (dccrg_cartesian_geometry.hpp:184) */
int dccrgx_set_geometry(dccrgx_grid* g, const double start[3], const double level_0_cell_length[3]);

/* Cartesian_Geometry::get_center / get_length (dccrg_cartesian_geometry.hpp:
 * 282-362) of n cells: 3 doubles per cell each (either output may be NULL);
 * NaN for invalid ids */
/* Cartesian_Geometry::get_start / get_level_0_cell_length (ABI 8); either
 * output may be NULL */
int dccrgx_get_geometry(dccrgx_grid* g, double start[3], double level_0_cell_length[3]);
/* The grid file's geometry block of a Stretched_Cartesian_Geometry
 * (Stretched_Cartesian_Geometry::write / read,
 * dccrg_stretched_cartesian_geometry.hpp:652-800: int id 2, 3 x uint64
 * coordinate counts, the coordinates as doubles), which save_grid_data then
 * writes instead of the Cartesian block (n = 0: the Cartesian block again);
 * DCCRGX_EINVAL for other bytes.  After load_grid_data of a file with such a
 * block, dccrgx_get_geometry_block returns it (*n = 0 for a Cartesian file;
 * out = NULL: the size only) and the library's own geometry takes each
 * dimension's start and first cell length (ABI 10). */
int dccrgx_set_geometry_block(dccrgx_grid* g, const void* bytes, size_t n);
int dccrgx_get_geometry_block(dccrgx_grid* g, void* out, size_t cap, size_t* n);
int dccrgx_geometry_batch(dccrgx_grid* g, const uint64_t* ids, size_t n, double* center, double* length);

/* ---- mapping (dccrg_mapping.hpp) — host-side scalar queries -------------- */
uint64_t dccrgx_get_cell_from_indices(dccrgx_grid* g, const uint64_t indices[3], int level); /* 153 */
int dccrgx_get_indices(dccrgx_grid* g, uint64_t cell, uint64_t indices[3]);                 /* 217 */
int dccrgx_get_refinement_level(dccrgx_grid* g, uint64_t cell);                             /* 261 */
uint64_t dccrgx_get_last_cell(dccrgx_grid* g);                                              /* 651 */
/* The same id math as the device kernels evaluate it, for n ids (valid
 * before initialize): level[i] (-1 for an invalid id) and 15 words per id in
 * out, following dccrg_mapping.hpp: indices x,y,z (get_indices 217), length
 * in indices (297), parent (get_parent 367), first child (get_child 338),
 * level-0 parent (479), siblings x8 (get_siblings 449); error_cell (0) in
 * every word of an invalid id. */
int dccrgx_mapping_batch(dccrgx_grid* g, const uint64_t* ids, size_t n, int32_t* level, uint64_t* out);

/* ---- queries ------------------------------------------------------------- */
/* get_cells(criteria={}, sorted=true) restricted to a selection; 651 */
int dccrgx_get_cells(dccrgx_grid* g, int which, uint64_t* out, size_t cap, size_t* n);
int dccrgx_get_counts(dccrgx_grid* g, size_t* n_inner, size_t* n_outer, size_t* n_recv, size_t* n_slots);
/* get_neighbors_of 819 (stencil order, error cells dropped as in 4634);
 * offsets as int32 x,y,z triples.  Returns DCCRGX_ENOTFOUND for non-local cells. */
int dccrgx_get_neighbors_of(dccrgx_grid* g, uint64_t cell, uint64_t* ids, int32_t* offsets, size_t cap, size_t* n);
/* all slot ids (slot order, see the layout above) */
int dccrgx_get_slot_ids(dccrgx_grid* g, uint64_t* out, size_t cap, size_t* n);
/* bulk download of a local CSR in slot order (rows = local slots):
 * kind 0 neighbors_of (aux = x,y,z offsets), 1 neighbors_to, 2 face
 * neighbors (aux = direction), 3 iterator cell.neighbors_of (update_cell_
 * pointers 11451-11500: only-of then both, each in (id, offset) order; aux
 * = x,y,z offsets).
 * ptr has n_local + 1 entries; *n = number of entries. */
int dccrgx_download_csr(dccrgx_grid* g, int kind, uint32_t* ptr, uint64_t* ids, int32_t* aux, size_t cap, size_t* n);
/* get_cells(criteria, exact_match, neighborhood_id, sorted=true) 651 with
 * is_neighbor_type_match 2946-3053: local cells whose neighbor types (the
 * bits has_local_neighbor_of 1, _to 2, has_remote_neighbor_of 4, _to 8 of
 * dccrg.hpp:95-142, from neighbors_of / neighbors_to of the neighborhood)
 * intersect the OR of the criteria (exact_match = 0) or equal one of them
 * (exact_match = 1); nc = 0 returns every local cell; ascending id */
int dccrgx_get_cells_by_criteria(dccrgx_grid* g, const int32_t* criteria, size_t nc, int exact_match, int hood_id,
                                 uint64_t* out, size_t cap, size_t* n);
/* slots of many cells (-1 when a cell has no slot on this rank) */
int dccrgx_get_slots(dccrgx_grid* g, const uint64_t* ids, size_t n, int64_t* slots);
/* bulk download of a user neighborhood's CSR in slot order (kind 0
 * neighbors_of with x,y,z offsets, 1 neighbors_to); as dccrgx_download_csr */
int dccrgx_download_user_csr(dccrgx_grid* g, int hood_id, int kind, uint32_t* ptr, uint64_t* ids, int32_t* offsets,
                             size_t cap, size_t* n);
/* get_neighbors_to 883 (ascending id, offsets 0) */
int dccrgx_get_neighbors_to(dccrgx_grid* g, uint64_t cell, uint64_t* ids, size_t cap, size_t* n);
/* get_face_neighbors_of 2806 (dirs -1,+1,-2,+2,-3,+3): a local cell from the
 * device face lists; a remote cell this process knows (e.g. a copy in
 * all_cells()) from its known leaves, DCCRGX_ENOTFOUND if one of its faces
 * lies beyond the ghost region */
int dccrgx_get_face_neighbors_of(dccrgx_grid* g, uint64_t cell, uint64_t* ids, int32_t* dirs, size_t cap, size_t* n);
/* is_local 3270, get_process 5807 (-1 for unknown cells) */
int dccrgx_is_local(dccrgx_grid* g, uint64_t cell);
int dccrgx_get_process(dccrgx_grid* g, uint64_t cell);
/* slot of a local cell or remote copy (-1 if none) */
int64_t dccrgx_get_slot(dccrgx_grid* g, uint64_t cell);
/* peers of this rank and their send/receive lists (cells_to_send /
 * cells_to_receive 6900-6914, 8590-8752; ascending id = wire order) */
int dccrgx_get_peers(dccrgx_grid* g, int32_t* peers, size_t cap, size_t* n);
int dccrgx_get_cells_to_send(dccrgx_grid* g, int peer, uint64_t* ids, size_t cap, size_t* n);
int dccrgx_get_cells_to_receive(dccrgx_grid* g, int peer, uint64_t* ids, size_t cap, size_t* n);
/* the leaves this rank knows with their processes, ascending id: its own
 * and its ghost leaves (the reference's get_cell_process 6848 returns every
 * leaf of the grid); ids == NULL: *n = count only */
int dccrgx_get_cell_process(dccrgx_grid* g, uint64_t* ids, int32_t* owners, size_t cap, size_t* n);

/* find_neighbors_of(cell, neighborhood) 4339-4680 for any list of n_items
 * offsets (3 x int32 each, cell-sized units): the (id, x/y/z offset) pairs in
 * item order, a finer box as its 8 cells in z-order, error cells dropped -
 * the sequence the reference's walk over the face cache produces.
 * DCCRGX_ENOTFOUND for a cell this process does not know (the reference
 * throws, 4354-4362).  For a local cell every item's box must lie within the
 * process's ghost region (max(neighborhood length, 1) level-0 cells around
 * the cell's level-0 parent; DCCRGX_EINVAL otherwise); for a remote cell the
 * list may be incomplete, as the reference documents (4327-4328). */
int dccrgx_find_neighbors_of(dccrgx_grid* g, uint64_t cell, const int32_t* items, size_t n_items, uint64_t* ids,
                             int32_t* offsets, size_t cap, size_t* n);
/* get_neighbors_ 7098-7109 (the face-neighbor cache of update_neighbors_
 * 9313-9458): per leaf the cell at the min corner just across each face,
 * directions -x,+x,-y,+y,-z,+z, error_cell (0) where none.  The reference
 * holds an entry for every leaf of the grid; here every known leaf whose six
 * probes land in level-0 cells this process knows (all own leaves and the
 * inner ghosts): n leaves ascending in ids, 6 x n entries in nbrs.  Costs
 * O(known leaves) on the host (a query for tests, not a sweep). */
int dccrgx_get_face_cache(dccrgx_grid* g, uint64_t* ids, uint64_t* nbrs, size_t cap, size_t* n);
/* unpin_all_cells 6017: drop every pin of this process (collective in the
 * reference; pins here are held by the process owning the cell) */
int dccrgx_unpin_all_cells(dccrgx_grid* g);

/* get_number_of_update_send_cells / _receive_cells 5382-5490 */
int dccrgx_get_number_of_update_cells(dccrgx_grid* g, uint64_t* n_send, uint64_t* n_receive);

/* ---- refinement (refine_completely 2434, unrefine_completely 2560,
 * dont_unrefine 2679, dont_refine 2744, stop_refining 3461 -> override_refines
 * 9991, induce_refines 9591, override_unrefines 9796, execute_refines 10104).
 * Requests are local leaves only (ENOTFOUND otherwise; unrefine_completely
 * also when a sibling has children).  stop_refining is collective: refined
 * leaves get their 8 children (owner and, here, payload inherited), merged
 * families become their parent (owner of the first child, payload zeroed);
 * the removed children's payloads move to the parent's process, where
 * get_removed_cells / dccrgx_removed_field_* expose them until the next
 * stop_refining or balance_load (unrefined_cell_data 7250, 3497). */
int dccrgx_refine_completely(dccrgx_grid* g, uint64_t cell);
int dccrgx_unrefine_completely(dccrgx_grid* g, uint64_t cell);
int dccrgx_dont_unrefine(dccrgx_grid* g, uint64_t cell);
int dccrgx_dont_refine(dccrgx_grid* g, uint64_t cell);
int dccrgx_stop_refining(dccrgx_grid* g, uint64_t* new_cells, size_t cap, size_t* n);
/* removed cells whose parent is local, in the order of the payload arrays
 * below (the kept children ascending, then per source rank ascending) */
int dccrgx_get_removed_cells(dccrgx_grid* g, uint64_t* ids, size_t cap, size_t* n);
/* a field's payloads of those cells: n x elem_bytes */
int dccrgx_removed_field_download(dccrgx_grid* g, int field_id, void* host, size_t cap_bytes);
int dccrgx_removed_field_device_ptr(dccrgx_grid* g, int field_id, void** ptr);
/* the local cells created by the last stop_refining (ascending) */
int dccrgx_get_new_cells(dccrgx_grid* g, uint64_t* new_cells, size_t cap, size_t* n);

/* Replace the whole leaf set and its partition (every rank passes the same
 * global list: ids strictly ascending, owners in [0, size)); the rank keeps
 * its own and its ghost leaves.  Setup path for a mesh + partition handed
 * over from outside (as load_grid_data 1089-2425 reads every cell's record);
 * payloads of cells that stay local are kept.  No communication. */
int dccrgx_set_cells(dccrgx_grid* g, const uint64_t* ids, const int32_t* owners, size_t n);

/* ---- user neighborhoods (add_neighborhood 6383-6520, remove_neighborhood
 * 6530-6570, get_neighbors_of/_to(cell, id) 819/883, the id's
 * cells_to_send / _receive, update_copies_of_remote_neighbors(id) 966).
 * Offsets: 3 x int32 per item, within the default neighborhood (face
 * offsets when its length is 0), never (0,0,0); a rejected set returns
 * DCCRGX_EINVAL where the reference returns false.  Identical calls on every
 * rank.  kind 0 = neighbors_of (offsets filled), 1 = neighbors_to. */
#define DCCRGX_DEFAULT_HOOD -0xDCC  /* default_neighborhood_id (dccrg.hpp:93) */
int dccrgx_add_neighborhood(dccrgx_grid* g, int id, const int32_t* offsets, size_t n);
int dccrgx_remove_neighborhood(dccrgx_grid* g, int id);
int dccrgx_get_user_neighbors(dccrgx_grid* g, int id, uint64_t cell, int kind, uint64_t* ids, int32_t* offsets,
                              size_t cap, size_t* n);
int dccrgx_get_user_update_list(dccrgx_grid* g, int id, int peer, int receive, uint64_t* ids, size_t cap, size_t* n);
int dccrgx_update_copies_of_remote_neighbors_hood(dccrgx_grid* g, int id);

/* ---- grid files (save_grid_data 1089-1740, load_grid_data 1742-2425;
 * layout 1104-1120).  save: every rank calls it with the same arguments;
 * rank 0 writes the header bytes at `offset`, every rank its cells' records
 * and data: per cell the payloads of the transferred fields in field order,
 * a fixed-size field's window (dccrgx_set_field_window; what the cell's
 * get_mpi_datatype describes) and a variable-size field's bytes of the cell.
 * load: on a created, not yet initialized grid whose transferred fields are
 * registered as at save time; initializes the grid from the file (length,
 * refinement level, neighborhood length, periodicity, geometry), creates the
 * file's cells with the level-0 block partition inherited by children, and
 * reads the local cells' payloads; a variable-size field (at most one) takes
 * the rest of each record after the fixed-size fields that follow it. */
int dccrgx_save_grid_data(dccrgx_grid* g, const char* path, uint64_t offset, const void* header, size_t header_bytes);
int dccrgx_load_grid_data(dccrgx_grid* g, const char* path, uint64_t offset, size_t header_bytes);
/* the split load (start_loading_grid_data 1795, continue_loading_grid_data
 * 2112, finish_loading_grid_data 2380), for records whose layout the caller
 * learns from their first bytes (tests/restart/variable_cell_data.cpp):
 * start initializes the grid and its cells as load does and reads no
 * payload; each continue reads the next bytes of every local cell's record
 * into one field and advances the cell's position past them - a fixed-size
 * field its window (sizes NULL), a variable-size field sizes[s] bytes for
 * local slot s (its cells take those sizes); a request beyond a record's end
 * returns DCCRGX_EINVAL.  bytes_left: per local slot, the unread bytes of its
 * record.  Nothing else may change the grid between start and finish.
 * save_grid_data does not truncate the file (the reference does not
 * either), so the last record of a file is bounded by the end of the file:
 * bytes after the grid data (an older, longer file at the same path, or the
 * caller's own) count toward that record's bytes_left. */
int dccrgx_start_loading_grid_data(dccrgx_grid* g, const char* path, uint64_t offset, size_t header_bytes);
int dccrgx_continue_loading_grid_data(dccrgx_grid* g, int field_id, const uint64_t* sizes);
int dccrgx_finish_loading_grid_data(dccrgx_grid* g);
int dccrgx_grid_file_bytes_left(dccrgx_grid* g, uint64_t* bytes);

/* ---- partition (pin 5832/5859, unpin 5909, balance_load 1024 and its
 * split form initialize_balance_load 3746 / continue_balance_load 3899 /
 * finish_balance_load 3942).  Collective.  The new owners (make_new_partition
 * 8349-8581) are, each overriding the one before: the native partitioner's
 * (use_partitioner != 0 and load balancing method "RCB", the reference's
 * default Zoltan method 7082: recursive coordinate bisection of the leaves by
 * their centers and weights, computed on the device - parity unpinned against
 * Zoltan, which is absent), an optional export list of this rank (local cells
 * and their new process, a partitioner's Zoltan_LB_Balance export list), and
 * the pins.  Method "NONE" or use_partitioner == 0: only exports and pins move
 * (balance_load(false)).  Cell weights are dropped (1011-1018).  continue
 * moves the payloads of every field (RCCL or the host exchange); finish
 * rebuilds every structure on the device, fetching the new ghost leaves from
 * their owners, and places the arrived payloads. */
int dccrgx_pin(dccrgx_grid* g, uint64_t cell, int process);
int dccrgx_unpin(dccrgx_grid* g, uint64_t cell);
int dccrgx_balance_load(dccrgx_grid* g, int use_partitioner);
int dccrgx_balance_load_to(dccrgx_grid* g, const uint64_t* cells, const int32_t* new_process, size_t n);
int dccrgx_initialize_balance_load(dccrgx_grid* g, int use_partitioner, const uint64_t* cells,
                                   const int32_t* new_process, size_t n);
/* the native partitioner's decision alone, no migration: every local cell
 * (ascending id) and its new process.  Collective. */
int dccrgx_make_new_partition(dccrgx_grid* g, uint64_t* cells, int32_t* new_process, size_t cap, size_t* n);
/* set_load_balancing_method 8223 ("RCB" default, "NONE"; other Zoltan methods
 * are EINVAL) / get_load_balancing_method 8228 (NUL-terminated into out) */
int dccrgx_set_load_balancing_method(dccrgx_grid* g, const char* method);
int dccrgx_get_load_balancing_method(dccrgx_grid* g, char* out, size_t cap);
/* set_cell_weight 6210 (local leaves; ENOTFOUND otherwise; children inherit
 * their parent's weight) / get_cell_weight 6244 (1 when unset, NaN for a
 * cell that is not a local leaf) */
int dccrgx_set_cell_weight(dccrgx_grid* g, uint64_t cell, double weight);
double dccrgx_get_cell_weight(dccrgx_grid* g, uint64_t cell);
int dccrgx_continue_balance_load(dccrgx_grid* g);
/* between initialize_ and finish_balance_load: the cells leaving to
 * (incoming = 0) or arriving from (incoming = 1) `peer`, ascending (the
 * reference's cells_to_send / cells_to_receive during a balance, 3746-3884) */
int dccrgx_get_migration_cells(dccrgx_grid* g, int peer, int incoming, uint64_t* ids, size_t cap, size_t* n);
int dccrgx_finish_balance_load(dccrgx_grid* g);
/* Explicit migration transport (instead of continue_balance_load): the
 * message to / from `peer` = for every field in field order, the payload of
 * each moving cell in ascending id.  pack after initialize, place before
 * finish; *_size gives both byte counts. */
int dccrgx_migration_message_size(dccrgx_grid* g, int peer, size_t* send_bytes, size_t* recv_bytes);
int dccrgx_migration_pack(dccrgx_grid* g, int peer, void* buf, size_t cap);
int dccrgx_migration_place(dccrgx_grid* g, int peer, const void* buf, size_t bytes);

/* ---- fields (replaces Cell_Data + get_mpi_datatype, dccrg_get_cell_datatype.hpp:40-340)
 * transfer != 0: the field is part of update_copies_of_remote_neighbors. */
int dccrgx_add_field(dccrgx_grid* g, const char* name, size_t elem_bytes, int transfer, int* field_id);
int dccrgx_set_field_transfer(dccrgx_grid* g, int field_id, int transfer);
/* the bytes of each element the halo carries: [offset, offset + bytes) (what
 * Cell_Data::get_mpi_datatype describes; default: the whole element) */
int dccrgx_set_field_window(dccrgx_grid* g, int field_id, size_t offset, size_t bytes);
/* the field's device array (slot order).  The pointer stays valid until the
 * next structural change (refinement, balance_load, loading a file).  Writes
 * made through it are seen by every call; the library's own bookkeeping of a
 * field's contents (e.g. dccrgx_get_live_neighbors' record that the list
 * field's inner rows are already zero) is reset only when this function is
 * called, so a program that writes through a pointer it fetched earlier
 * fetches it again after such writes. */
int dccrgx_field_device_ptr(dccrgx_grid* g, int field_id, void** ptr);
/* host <-> device copies of whole slot ranges [slot0, slot0+n) */
int dccrgx_field_upload(dccrgx_grid* g, int field_id, size_t slot0, size_t n, const void* host);
int dccrgx_field_download(dccrgx_grid* g, int field_id, size_t slot0, size_t n, void* host);

/* ---- variable-size payloads (a Cell_Data whose get_mpi_datatype describes
 * a different number of bytes per cell, e.g. a std::vector member:
 * tests/variable_data_size/variable_data_size.cpp, variable_neighbour_data.cpp;
 * dccrg_get_cell_datatype.hpp:40-340).  One byte pool over all slots; a new
 * field, new children and new remote copies start empty (the reference
 * default-constructs them).  The halo, migrations (continue_balance_load)
 * and the removed-cell store move every cell's size with its bytes, so a
 * receiver takes the sender's sizes (the reference needs the receiver to
 * size its copies first, variable_neighbour_data.cpp:95-102, 133-145; done
 * that way the bytes are the same).  Grid files and the explicit halo /
 * migration message calls (dccrgx_halo_*, dccrgx_migration_*) refuse them
 * (DCCRGX_EINVAL); the fixed-field calls (dccrgx_field_*) refuse a variable
 * field. */
int dccrgx_add_variable_field(dccrgx_grid* g, const char* name, int transfer, int* field_id);
/* byte sizes of slots [slot0, slot0 + n) */
int dccrgx_variable_field_sizes(dccrgx_grid* g, int field_id, size_t slot0, size_t n, uint64_t* sizes);
/* new byte sizes of slots [slot0, slot0 + n): each cell keeps its first
 * min(old, new) bytes, new bytes are zero (std::vector::resize) */
int dccrgx_variable_field_resize(dccrgx_grid* g, int field_id, size_t slot0, size_t n, const uint64_t* sizes);
/* the concatenated bytes of slots [slot0, slot0 + n); upload needs exactly
 * their current total, download sets *nbytes (DCCRGX_ERANGE when cap is short) */
int dccrgx_variable_field_upload(dccrgx_grid* g, int field_id, size_t slot0, size_t n, const void* bytes,
                                 size_t nbytes);
int dccrgx_variable_field_download(dccrgx_grid* g, int field_id, size_t slot0, size_t n, void* bytes, size_t cap,
                                   size_t* nbytes);
/* device pool and the n_slots + 1 byte offsets (slot s: [off[s], off[s+1])) */
int dccrgx_variable_field_device_ptr(dccrgx_grid* g, int field_id, void** data, const uint64_t** offsets);
/* the removed cells' payloads (order of dccrgx_get_removed_cells): sizes
 * (one per removed cell, may be NULL) and concatenated bytes */
int dccrgx_removed_variable_field_download(dccrgx_grid* g, int field_id, uint64_t* sizes, void* bytes, size_t cap,
                                           size_t* nbytes);
/* set_send_single_cells 6677 / get_send_single_cells 6684: one message per
 * cell (tag = position + 1) instead of one per process.  On, the remote
 * neighbor updates put each cell's fixed-size payload on the wire as its own
 * message (per cell in the send list's order, a cell's fields in field
 * order; RCCL posts them in that order, which is how its point-to-point
 * matches them); off, one message per peer and field.  Variable-size fields,
 * migrations and removed-cell payloads keep one message per peer.  The
 * received payloads are identical either way. */
int dccrgx_set_send_single_cells(dccrgx_grid* g, int on);
int dccrgx_get_send_single_cells(dccrgx_grid* g, int* on);

/* ---- halo (update_copies_of_remote_neighbors 966-1000 and its split form
 * start_remote_neighbor_copy_updates 5010, wait_* 5267-5367) ------------- */
int dccrgx_update_copies_of_remote_neighbors(dccrgx_grid* g);
int dccrgx_start_remote_neighbor_copy_updates(dccrgx_grid* g);
int dccrgx_wait_remote_neighbor_copy_update_receives(dccrgx_grid* g);
int dccrgx_wait_remote_neighbor_copy_update_sends(dccrgx_grid* g);
int dccrgx_wait_remote_neighbor_copy_updates(dccrgx_grid* g);
/* Explicit halo transport of one neighborhood (DCCRGX_DEFAULT_HOOD or a user
 * id): the message to / from `peer` = for every transferred field in field
 * order, the window bytes of each cell of cells_to_send / cells_to_receive
 * in ascending id (the wire order of start_user_data_sends / _receives
 * 10587-10997).  pack gathers from the device fields into a host buffer,
 * place scatters a received message into the halo copies. */
int dccrgx_halo_message_size(dccrgx_grid* g, int hood_id, int peer, size_t* send_bytes, size_t* recv_bytes);
int dccrgx_halo_pack(dccrgx_grid* g, int hood_id, int peer, void* buf, size_t cap);
int dccrgx_halo_place(dccrgx_grid* g, int hood_id, int peer, const void* buf, size_t bytes);

/* ---- built-in sweeps (user stencils of tests/ and examples/) ------------- */
/* game of life over cell.neighbors_of (examples/game_of_life.cpp:54-79,
 * tests/game_of_life/scalability3d.cpp:130-165); state is a uint32 field.
 * Reads state, writes the next state into a scratch buffer; the field's
 * device pointer is swapped when dccrgx_gol_commit is called. */
int dccrgx_gol_step(dccrgx_grid* g, int state_field, int region);
int dccrgx_gol_commit(dccrgx_grid* g, int state_field);

/* Game of life on a refined grid emulating the unrefined game:
 * get_live_neighbors, tests/game_of_life/solve.hpp:37-170, split at its halo.
 * phase 0 (collect, 46-110): list_field[cell] = the distinct level-0 parents
 * of live neighbors (neighbors_of order, own parent skipped), error_cell (0)
 * padded; phase 1 (spread + rule, 113-167): merge the lists of same-parent
 * neighbors, count, update state in place.  Between the phases the caller
 * runs update_copies_of_remote_neighbors (both fields transferred).
 * list_field: 64-byte elements (8 x uint64 = Cell_Data::data[1..8]).
 * DCCRGX_EINVAL where the reference aborts (list overflow, siblings
 * disagreeing on their state). */
int dccrgx_gol_amr(dccrgx_grid* g, int phase, int state_field, int list_field, int region);
/* One whole turn of get_live_neighbors (solve.hpp:37-170): collect, the halo
 * (update_copies_of_remote_neighbors, every transferred field), spread + rule,
 * and every local list left error_cell-cleared as the reference's rule loop
 * leaves it (163).  Inside the turn the collected lists live in the kernels'
 * per-cell bit masks; list_field receives only the lists other processes
 * read (the outer cells'), for the halo, and those are cleared at the end.
 * Same states as phase 0 + halo + phase 1; same errors. */
int dccrgx_get_live_neighbors(dccrgx_grid* g, int state_field, int list_field);
/* first-order upwind advection over face neighbors, flux + apply fused
 * (tests/advection/solve.hpp:44-279).  fields: density, vx, vy, vz, lx, ly, lz
 * (all fp64).  Writes the new density into a scratch buffer; commit swaps. */
int dccrgx_advection_step(dccrgx_grid* g, const int fields[7], double dt, int region);
int dccrgx_advection_commit(dccrgx_grid* g, int density_field);
/* advection helpers: initial condition (tests/advection/initialize.hpp:36-82)
 * and max_time_step (solve.hpp:289-333, local part; caller reduces MIN) */
int dccrgx_advection_initialize(dccrgx_grid* g, const int fields[7]);
int dccrgx_advection_max_time_step(dccrgx_grid* g, const int fields[7], double* local_min);
/* the same, reduced over all processes (MIN in rank order, solve.hpp:317),
 * written to DEVICE memory d_out[0] in stream order on the compute stream:
 * no host synchronization over RCCL, so an adaptive loop can take dt
 * without a round trip (ABI 8) */
int dccrgx_advection_max_time_step_device(dccrgx_grid* g, const int fields[7], double* d_out);
/* refine candidates of check_for_adaptation (tests/advection/adapter.hpp:47-178):
 * local cells whose max face relative difference exceeds (lvl+1)*diff_increase */
int dccrgx_advection_refine_candidates(dccrgx_grid* g, int density_field, double diff_increase,
                                       double diff_threshold, uint64_t* out, size_t cap, size_t* n);

/* grid adaptation of tests/advection (adapter.hpp): check_adaptation
 * (47-178) classifies every local cell by the relative density difference to
 * its face neighbors and issues the refine / dont_unrefine / unrefine
 * requests adapt_grid would (counts: the three numbers accepted); call it
 * between the step and the commit, as 2d.cpp does before apply_fluxes.
 * adapt (232-309, collective): stop_refining, merged parents get their
 * children's mean density, velocities and lengths of every local cell are
 * reset, and all seven fields go through one halo (transfer_all_data).
 * out: created and removed cells of this rank. */
int dccrgx_advection_check_adaptation(dccrgx_grid* g, int density_field, double diff_increase,
                                      double diff_threshold, double unrefine_sensitivity, uint64_t counts[3]);
int dccrgx_advection_adapt(dccrgx_grid* g, const int fields[7], uint64_t out[2]);
/* data layout of the advection sweep (built on first use): out[0] tile size,
 * [1] tiles, [2] distinct out-of-tile face neighbors summed over the tiles,
 * [3] largest per-tile count, [4] finer faces, [5] face-neighbor entries
 * (get_face_neighbors_of summed over local cells), [6] algorithmic HBM bytes
 * of one sweep over all local cells as SURVEY §8(d) fixes them (64 B per cell
 * + 4 B per face entry + 4 B per row pointer), [7] the 64 B-per-cell core
 * alone, [8] regular tiles (aligned uniform boxes swept without face rows),
 * [9] cells in regular tiles, [10] out-of-tile face neighbors of the regular
 * tiles (64 per existing side), [11] the bytes the sweep kernels need per
 * sweep, each value read once: the 64-B core, per cell of an irregular tile
 * its 12 B of face codes, per out-of-tile neighbor its density, three
 * lengths and the velocity along the face (40 B; 32 B with the experimental
 * neighbor records) plus 4 B of list entry in an irregular tile, 8 B per
 * finer face, 32 B per tile record (ABI 9: out[12]).
 * No reference counterpart (roofline introspection). */
int dccrgx_advection_layout(dccrgx_grid* g, uint64_t out[12]);

/* ---- Poisson solver (tests/poisson/poisson_solve.hpp:156-1056) ----------
 * dccrgx_poisson_cache = Poisson_Solve::cache_system_info (827-971): local
 * cells default to boundary cells, ids in skip_cells are skipped, ids in
 * solve_cells are solved (non-local ids are ignored, as the reference does);
 * computes the geometry factors (set_scaling_factor 696-819) on the device and
 * halos them.  rhs / solution are fp64 fields.
 * dccrgx_poisson_solve = Poisson_Solve::solve (251-522, failsafe = 0) or
 * solve_failsafe (531-634, failsafe = 1) with the constructor's parameters
 * (187-201); solution = best solution on return.  *iterations = iterations
 * done, *residual = smallest residual (solve) or last norm (failsafe).
 * dccrgx_poisson_field: the solver's per-cell state as a field ("p0", "p1",
 * "r0", "r1", "A_dot_p0", "best_solution", "scaling_factor", "f_x_neg" ...
 * "f_z_pos", "type"), e.g. for inspection after a solve. */
int dccrgx_poisson_cache(dccrgx_grid* g, int rhs_field, int solution_field, const uint64_t* solve_cells,
                         size_t n_solve, const uint64_t* skip_cells, size_t n_skip);
int dccrgx_poisson_solve(dccrgx_grid* g, unsigned max_iterations, unsigned min_iterations, double stop_residual,
                         double p_of_norm, double stop_after_residual_increase, int failsafe, unsigned* iterations,
                         double* residual);
int dccrgx_poisson_field(dccrgx_grid* g, const char* name, int* field_id);

/* ---- collectives for user kernels (MPI_Allreduce in solve.hpp:317) ------- */
int dccrgx_allreduce_f64(dccrgx_grid* g, double* inout, int count, int op /* 0 sum, 1 min, 2 max */);
/* MPI_Allreduce on DEVICE doubles (dccrg_mpi_support.hpp All_Reduce's role
 * for fp64), queued on the compute stream: the processes' values are
 * all-gathered on the device and combined in rank order by one kernel, so
 * the result is bitwise dccrgx_allreduce_f64's and, over RCCL, nothing waits
 * on the host (a host exchange transport stages through the host).  d_in may
 * equal d_out (ABI 8) */
int dccrgx_allreduce_f64_device(dccrgx_grid* g, const double* d_in, double* d_out, int count, int op);
int dccrgx_barrier(dccrgx_grid* g);

/* The transport the grid was built on (no reference counterpart; the
 * reference's MPI_Comm_size on its duplicated communicator): *kind is
 * DCCRGX_TRANSPORT_NONE (a detached view), _RCCL or _HOST (an exchange
 * function), *comm_ranks the ranks of the communicator the library holds -
 * ncclCommCount of its RCCL communicator, the grid's size for a host exchange,
 * 1 for a detached view (ABI 9) */
#define DCCRGX_TRANSPORT_NONE 0
#define DCCRGX_TRANSPORT_RCCL 1
#define DCCRGX_TRANSPORT_HOST 2
int dccrgx_get_transport(dccrgx_grid* g, int* kind, int* comm_ranks);

/* Transport check (no reference counterpart): the bytes of a fixed-size
 * field's slots [slot0, slot0 + n) sent by this process to itself and
 * received straight into slots [dst_slot0, dst_slot0 + n) of the same field,
 * through the grid's RCCL byte mover (one grouped ncclSend / ncclRecv, the
 * path of every halo and migration message; a grid created with an RCCL id,
 * also at size 1).  Under send_single_cells the n elements go out as n
 * messages, as a halo's cells do (ABI 9).  DCCRGX_EINVAL on a host-exchange
 * or detached grid. */
int dccrgx_comm_loopback(dccrgx_grid* g, int field_id, size_t slot0, size_t n, size_t dst_slot0);

/* ---- stream / timing ----------------------------------------------------- */
int dccrgx_synchronize(dccrgx_grid* g);
void* dccrgx_compute_stream(dccrgx_grid* g);
/* average duration (ms) of the last `count` sweep kernels measured with HIP
 * events on the compute stream; enable=1 starts recording */
int dccrgx_kernel_timing(dccrgx_grid* g, int enable, double* total_ms, int64_t* count);

#ifdef __cplusplus
}
#endif

#endif /* DCCRGX_H */
