// BASELINE config 1's driver (reference examples/game_of_life.cpp: 500 x
// 500 x 1, neighborhood 1) written against the drop-in facade with the
// per-cell loops on the GPU: the state is a device SoA field swept by the
// library's game of life, with the reference's start / inner / wait / outer
// / apply overlap.  Any number of MPI ranks (RCCL when each has a GPU, the
// MPI host exchange otherwise).
//
// usage: mpiexec -n P game_of_life [turns]
//   prints on rank 0: "cells <N> turns <T> live <L> rate <cell-updates/s>"
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mpi.h"

#include "dccrg.hpp"

struct game_of_life_cell {
	unsigned int is_alive = 0, live_neighbor_count = 0;
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() {
		return std::make_tuple((void*)&is_alive, 1, MPI_UNSIGNED);
	}
};

static uint32_t alive0(uint64_t id) {  // seeded, independent of the partition
	uint64_t z = (id ^ 0x5DEECE66Dull) + 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	z = z ^ (z >> 31);
	return z < uint64_t(0.2 * 18446744073709551616.0) ? 1u : 0u;
}

int main(int argc, char* argv[])
{
	MPI_Init(&argc, &argv);
	const int turns = argc > 1 ? std::atoi(argv[1]) : 100;
	uint64_t total = 0, live = 0;
	double seconds = 0;
	int rank = 0;
	{
		dccrg::Dccrg<game_of_life_cell> grid;
		grid.set_initial_length({500, 500, 1}).set_neighborhood_length(1).set_maximum_refinement_level(0);
		grid.set_host_staging(false);  // the state lives in a device field, not in Cell_Data
		grid.initialize(MPI_COMM_WORLD);
		rank = grid.get_rank();
		// the state as a device field (facade members, no raw C calls)
		const auto state = grid.add_field<uint32_t>("is_alive", true);
		const auto slots = grid.get_slot_ids();
		std::vector<uint32_t> alive(grid.get_number_of_local_slots());
		for (size_t s = 0; s < alive.size(); s++) alive[s] = alive0(slots[s]);
		state.set(alive);

		MPI_Barrier(MPI_COMM_WORLD);
		const auto t0 = std::chrono::high_resolution_clock::now();
		for (int turn = 0; turn < turns; turn++) {
			grid.start_remote_neighbor_copy_updates();
			grid.gol_step(state, DCCRGX_REGION_INNER);
			grid.wait_remote_neighbor_copy_update_receives();
			grid.gol_step(state, DCCRGX_REGION_OUTER);
			grid.wait_remote_neighbor_copy_update_sends();
			grid.gol_commit(state);
		}
		grid.synchronize();
		MPI_Barrier(MPI_COMM_WORLD);
		seconds = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
		alive = state.get(alive.size());
		uint64_t mine = 0, n = alive.size();
		for (auto a : alive) mine += a;
		MPI_Reduce(&mine, &live, 1, MPI_UINT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
		MPI_Reduce(&n, &total, 1, MPI_UINT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
	}
	if (rank == 0)
		std::printf("cells %llu turns %d live %llu rate %.4e\n", (unsigned long long)total, turns,
		            (unsigned long long)live, double(total) * turns / seconds);
	MPI_Finalize();
	return 0;
}
