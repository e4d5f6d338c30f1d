/*
 * dccrg_mpi_support.hpp - the facade's MPI helpers with the reference's names
 * and meanings (reference dccrg_mpi_support.hpp:40-380), which test programs
 * written against dccrg use directly (e.g. tests/refine/dont_refine.cpp's
 * All_Reduce).  Plain MPI calls; a failing call aborts, as in the reference.
 */
#ifndef DCCRG_AMD_MPI_SUPPORT_HPP
#define DCCRG_AMD_MPI_SUPPORT_HPP

#include <mpi.h>

#include <cstdint>
#include <cstdlib>
#include <iostream>
#include <string>
#include <unordered_set>
#include <vector>

namespace dccrg {

// 40-57: the text of an MPI error code
class Error_String {
public:
	std::string operator()(int mpi_return_value) {
		char text[MPI_MAX_ERROR_STRING + 1] = {0};
		int n = 0;
		MPI_Error_string(mpi_return_value, text, &n);
		return std::string(text, size_t(n > 0 ? n : 0));
	}
};

// 63-92: whether a datatype is one of MPI's predefined (named) types
class Is_Named_Datatype {
public:
	bool operator()(MPI_Datatype& type) const {
		int ni = -1, na = -1, nd = -1, combiner = -1;
		const int rc = MPI_Type_get_envelope(type, &ni, &na, &nd, &combiner);
		if (rc != MPI_SUCCESS) {
			std::cerr << __FILE__ << ":" << __LINE__ << " MPI_Type_get_envelope failed: " << Error_String()(rc)
			          << std::endl;
			abort();
		}
		return combiner == MPI_COMBINER_NAMED;
	}
};

// 98-231: every process's uint64 values, result[p] = the values of process p
class All_Gather {
public:
	void operator()(std::vector<uint64_t>& values, std::vector<std::vector<uint64_t>>& result, MPI_Comm& comm) {
		int size = 0;
		MPI_Comm_size(comm, &size);
		if (values.size() > size_t(INT32_MAX)) {
			std::cerr << __FILE__ << ":" << __LINE__ << " Tried to send more values than INT_MAX." << std::endl;
			abort();
		}
		int mine = int(values.size());
		std::vector<int> counts(size_t(size), 0), displ(size_t(size), 0);
		if (MPI_Allgather(&mine, 1, MPI_INT, counts.data(), 1, MPI_INT, comm) != MPI_SUCCESS) abort();
		size_t total = 0;
		for (int p = 0; p < size; p++) {
			displ[size_t(p)] = int(total);
			total += size_t(counts[size_t(p)]);
		}
		std::vector<uint64_t> all(total + 1);
		uint64_t dummy = 0;
		if (MPI_Allgatherv(values.empty() ? &dummy : values.data(), mine, MPI_UINT64_T, all.data(), counts.data(),
		                   displ.data(), MPI_UINT64_T, comm) != MPI_SUCCESS)
			abort();
		result.assign(size_t(size), {});
		for (int p = 0; p < size; p++)
			result[size_t(p)].assign(all.begin() + displ[size_t(p)], all.begin() + displ[size_t(p)] + counts[size_t(p)]);
	}
};

// 237-266: the sum of a uint64 over all processes
class All_Reduce {
public:
	uint64_t operator()(uint64_t value, MPI_Comm& comm) {
		uint64_t result = 0;
		const int rc = MPI_Allreduce(&value, &result, 1, MPI_UINT64_T, MPI_SUM, comm);
		if (rc != MPI_SUCCESS) {
			std::cerr << __FILE__ << ":" << __LINE__ << " MPI_Allreduce failed: " << Error_String()(rc) << std::endl;
			abort();
		}
		return result;
	}
};

// 282-380: the sum of a uint64 over this process and the given neighbor
// processes only (each pair must list each other)
class Some_Reduce {
public:
	uint64_t operator()(uint64_t value, const std::unordered_set<int>& neighbors, MPI_Comm& comm) {
		std::vector<int> peers(neighbors.begin(), neighbors.end());
		std::vector<uint64_t> got(peers.size(), 0);
		std::vector<MPI_Request> req(2 * peers.size());
		for (size_t i = 0; i < peers.size(); i++)
			if (MPI_Irecv(&got[i], 1, MPI_UINT64_T, peers[i], 1, comm, &req[i]) != MPI_SUCCESS) abort();
		for (size_t i = 0; i < peers.size(); i++)
			if (MPI_Isend(&value, 1, MPI_UINT64_T, peers[i], 1, comm, &req[peers.size() + i]) != MPI_SUCCESS) abort();
		if (!req.empty() && MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE) != MPI_SUCCESS) abort();
		uint64_t r = value;
		for (const uint64_t v : got) r += v;
		return r;
	}
};

}  // namespace dccrg

#endif
