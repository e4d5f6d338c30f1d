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
		grid.initialize(MPI_COMM_WORLD);
		rank = grid.get_rank();
		dccrgx_grid* g = grid.native();
		const int state = grid.add_field<uint32_t>("is_alive", true);
		// the device field in slot order
		const auto slots = dccrg::detail::fetch_u64([&](uint64_t* o, size_t c, size_t* n) {
			return dccrgx_get_slot_ids(g, o, c, n);
		});
		size_t ni = 0, no = 0;
		dccrg::detail::check(dccrgx_get_counts(g, &ni, &no, nullptr, nullptr));
		std::vector<uint32_t> alive(ni + no);
		for (size_t s = 0; s < alive.size(); s++) alive[s] = alive0(slots[s]);
		dccrg::detail::check(dccrgx_field_upload(g, state, 0, alive.size(), alive.data()));

		MPI_Barrier(MPI_COMM_WORLD);
		const auto t0 = std::chrono::high_resolution_clock::now();
		for (int turn = 0; turn < turns; turn++) {
			dccrg::detail::check(dccrgx_start_remote_neighbor_copy_updates(g));
			dccrg::detail::check(dccrgx_gol_step(g, state, DCCRGX_REGION_INNER));
			dccrg::detail::check(dccrgx_wait_remote_neighbor_copy_update_receives(g));
			dccrg::detail::check(dccrgx_gol_step(g, state, DCCRGX_REGION_OUTER));
			dccrg::detail::check(dccrgx_wait_remote_neighbor_copy_update_sends(g));
			dccrg::detail::check(dccrgx_gol_commit(g, state));
		}
		dccrg::detail::check(dccrgx_synchronize(g));
		MPI_Barrier(MPI_COMM_WORLD);
		seconds = std::chrono::duration<double>(std::chrono::high_resolution_clock::now() - t0).count();
		dccrg::detail::check(dccrgx_field_download(g, state, 0, alive.size(), alive.data()));
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
