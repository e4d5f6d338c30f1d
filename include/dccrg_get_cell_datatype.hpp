/*
 * dccrg_get_cell_datatype.hpp - the facade's dccrg::detail::get_cell_mpi_datatype
 * (reference dccrg_get_cell_datatype.hpp:40-340): the (address, count,
 * MPI_Datatype) a cell hands to a transfer.
 *
 * Overload rules kept from the reference (tests/get_cell_datatype/run_time.cpp
 * and get_cell_mpi_datatype.cpp check them):
 *   - a member get_mpi_datatype(cell, sender, receiver, receiving, hood) is
 *     preferred over the zero-argument one, each matched with the object's own
 *     constness (a const member is found through a const reference, a non-const
 *     member through a non-const reference, and overload resolution prefers the
 *     non-const binding);
 *   - without a member, the standard arithmetic types and std::array of them map
 *     to their named MPI type with count 1 (array: its size).
 * Detection of an exact member signature uses a static_cast to the member
 * function pointer type (no Boost).  Unlike the reference, a type with no
 * member and no named MPI type is sent as its raw bytes (the reference stops
 * with a static_assert).
 */
#ifndef DCCRG_AMD_GET_CELL_DATATYPE_HPP
#define DCCRG_AMD_GET_CELL_DATATYPE_HPP

#include <mpi.h>

#include <array>
#include <cstddef>
#include <cstdint>
#include <tuple>
#include <type_traits>

namespace dccrg {
namespace detail {

using mpi_transfer_t = std::tuple<void*, int, MPI_Datatype>;

// exact member signatures, the reference's four BOOST_TTI checks
template <class T, class = void>
struct has_dt5_const : std::false_type {};
template <class T>
struct has_dt5_const<T, decltype((void)static_cast<mpi_transfer_t (T::*)(uint64_t, int, int, bool, int) const>(
                            &T::get_mpi_datatype))> : std::true_type {};
template <class T, class = void>
struct has_dt5 : std::false_type {};
template <class T>
struct has_dt5<T, decltype((void)static_cast<mpi_transfer_t (T::*)(uint64_t, int, int, bool, int)>(
                      &T::get_mpi_datatype))> : std::true_type {};
template <class T, class = void>
struct has_dt0_const : std::false_type {};
template <class T>
struct has_dt0_const<T, decltype((void)static_cast<mpi_transfer_t (T::*)() const>(&T::get_mpi_datatype))>
    : std::true_type {};
template <class T, class = void>
struct has_dt0 : std::false_type {};
template <class T>
struct has_dt0<T, decltype((void)static_cast<mpi_transfer_t (T::*)()>(&T::get_mpi_datatype))> : std::true_type {};

template <class T>
struct has_any_datatype_member
    : std::integral_constant<bool, has_dt5_const<T>::value || has_dt5<T>::value || has_dt0_const<T>::value ||
                                       has_dt0<T>::value> {};

// the named types (reference 226-281)
#define DCCRGX_BASIC_DATATYPE(CPP, MPI)                                            \
	inline mpi_transfer_t get_mpi_datatype_basic(CPP& cell) {                      \
		return std::make_tuple(static_cast<void*>(&cell), 1, MPI);                  \
	}                                                                              \
	template <size_t N>                                                            \
	inline mpi_transfer_t get_mpi_datatype_basic(std::array<CPP, N>& cell) {       \
		return std::make_tuple(static_cast<void*>(cell.data()), int(N), MPI);       \
	}
DCCRGX_BASIC_DATATYPE(char, MPI_CHAR)
DCCRGX_BASIC_DATATYPE(signed char, MPI_CHAR)
DCCRGX_BASIC_DATATYPE(unsigned char, MPI_UNSIGNED_CHAR)
DCCRGX_BASIC_DATATYPE(short int, MPI_SHORT)
DCCRGX_BASIC_DATATYPE(unsigned short int, MPI_UNSIGNED_SHORT)
DCCRGX_BASIC_DATATYPE(int, MPI_INT)
DCCRGX_BASIC_DATATYPE(unsigned int, MPI_UNSIGNED)
DCCRGX_BASIC_DATATYPE(long int, MPI_LONG)
DCCRGX_BASIC_DATATYPE(unsigned long int, MPI_UNSIGNED_LONG)
DCCRGX_BASIC_DATATYPE(long long int, MPI_LONG_LONG)
DCCRGX_BASIC_DATATYPE(unsigned long long int, MPI_UNSIGNED_LONG_LONG)
DCCRGX_BASIC_DATATYPE(float, MPI_FLOAT)
DCCRGX_BASIC_DATATYPE(double, MPI_DOUBLE)
DCCRGX_BASIC_DATATYPE(long double, MPI_LONG_DOUBLE)
DCCRGX_BASIC_DATATYPE(wchar_t, MPI_WCHAR)
#undef DCCRGX_BASIC_DATATYPE
inline mpi_transfer_t get_mpi_datatype_basic(bool& cell) {
	return std::make_tuple(static_cast<void*>(&cell), 1, MPI_CXX_BOOL);
}
// any other type without a member: its bytes
template <class T>
mpi_transfer_t get_mpi_datatype_basic(T& cell) {
	return std::make_tuple(const_cast<void*>(static_cast<const void*>(&cell)), int(sizeof(T)), MPI_BYTE);
}

// five-argument members (reference 48-125)
template <class T>
typename std::enable_if<has_dt5_const<T>::value, mpi_transfer_t>::type get_cell_mpi_datatype(
    const T& cell, const uint64_t cell_id, const int sender, const int receiver, const bool receiving,
    const int neighborhood_id) {
	return cell.get_mpi_datatype(cell_id, sender, receiver, receiving, neighborhood_id);
}
template <class T>
typename std::enable_if<!std::is_const<T>::value && has_dt5<T>::value, mpi_transfer_t>::type get_cell_mpi_datatype(
    T& cell, const uint64_t cell_id, const int sender, const int receiver, const bool receiving,
    const int neighborhood_id) {
	return cell.get_mpi_datatype(cell_id, sender, receiver, receiving, neighborhood_id);
}
// zero-argument members, each only when the same constness has no
// five-argument member (reference 134-213)
template <class T>
typename std::enable_if<has_dt0_const<T>::value && !has_dt5_const<T>::value, mpi_transfer_t>::type
get_cell_mpi_datatype(const T& cell, const uint64_t, const int, const int, const bool, const int) {
	return cell.get_mpi_datatype();
}
template <class T>
typename std::enable_if<!std::is_const<T>::value && has_dt0<T>::value && !has_dt5<T>::value, mpi_transfer_t>::type
get_cell_mpi_datatype(
    T& cell, const uint64_t, const int, const int, const bool, const int) {
	return cell.get_mpi_datatype();
}
// no member at all (reference 288-339)
template <class T>
typename std::enable_if<!has_any_datatype_member<T>::value, mpi_transfer_t>::type get_cell_mpi_datatype(
    T& cell, const uint64_t, const int, const int, const bool, const int) {
	return get_mpi_datatype_basic(cell);
}

}  // namespace detail
}  // namespace dccrg

#endif
