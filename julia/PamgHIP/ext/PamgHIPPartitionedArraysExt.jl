# PamgHIPPartitionedArraysExt — PartitionedArrays.jl (v0.5 API) adapter of PamgHIP.
#
# An AMG solver written against PartitionedArrays keeps calling mul!, consistent!, dot, norm,
# axpy!, ldiv! on PSparseMatrix / PVector; this extension moves the parts onto the GPU(s) once
# (`hip(A)`, `hip(x)`) and gives those calls device methods that run libpamg's kernels:
#
#   A_d = hip(ctxs, A)            # PSparseMatrix -> HIPPSparseMatrix (one DeviceMatrix per part)
#   x_d = hip(ctxs, x)            # PVector       -> HIPPVector       (own + ghost slots per part)
#   mul!(y_d, A_d, x_d)           # ghost exchange (RCCL / debug transport) + SpMV per part
#   t = consistent!(x_d); wait(t) # split exchange (pamg_exchange_begin / _end)
#   copyto!(x, x_d)               # own values back into the PartitionedArrays vector
#
# `ctxs` is a PartitionedArrays array of PamgHIP.Context, one per part, made with `map` over
# the parts (with_mpi: one rank = one part = one GPU, each context comm_init!'ed; with_debug:
# all parts in one process, e.g. Context(0) for each, no communicator).
#
# Layout mapping. PartitionedArrays numbers a part's local indices own-first for the
# OwnAndGhostIndices it builds (uniform_partition + ghosts), with ghosts in the order of
# ghost_to_global. libpamg wants the ghosts grouped by owner, in neighbour order (SPEC §S7,
# include/pamg.h pamg_plan_create). `DeviceLayout` records the permutation: device ghost slot
# j holds PartitionedArrays local index `ghost_lids[j]`; matrix columns are renumbered with it
# at upload and vectors are permuted on the way in and out. Send lists are the owners' local
# indices of the ghosts each neighbour holds, obtained with PartitionedArrays' own `exchange`.
module PamgHIPPartitionedArraysExt

using LinearAlgebra
using SparseArrays
using PartitionedArrays
using PamgHIP
import PamgHIP: DeviceVector, DeviceMatrix, ExchangePlan, Context, own_values, consistent!

# ------------------------------------------------------------------ layout of one part
struct DeviceLayout
    n_own::Int
    own_lids::Vector{Int32}       # PartitionedArrays local ids of the own entries, device order
    ghost_lids::Vector{Int32}     # ... of the ghost entries, device slot order
    lid_to_device::Vector{Int32}  # PartitionedArrays local id -> device local id (1-based)
    nbr_ranks::Vector{Int32}      # 0-based ranks, device neighbour order
    recv_counts::Vector{Int64}
end

function device_layout(ids)
    own = Int32.(collect(own_to_local(ids)))
    gl = collect(ghost_to_local(ids))
    owner = collect(ghost_to_owner(ids))
    # ghosts grouped by owner (ascending part id), original order within a group (stable)
    perm = sortperm(owner; alg = Base.Sort.DEFAULT_STABLE)
    ghost_lids = Int32.(gl[perm])
    nbrs = unique(owner[perm])
    counts = Int64[count(==(q), owner) for q in nbrs]
    l2d = zeros(Int32, local_length(ids))
    for (k, l) in enumerate(own)
        l2d[l] = k
    end
    for (k, l) in enumerate(ghost_lids)
        l2d[l] = length(own) + k
    end
    DeviceLayout(length(own), own, ghost_lids, l2d, Int32.(nbrs .- 1), counts)
end

"""
Per-part exchange plans for the index partition `rows` (a PRange's `partition`): each part
asks the owners of its ghosts (in device order) for them through PartitionedArrays'
`exchange`, and the answers are the owners' send lists.
"""
function exchange_plans(ctxs, rows, layouts)
    parts = linear_indices(rows)
    # requests: for every neighbour, the global ids of the ghosts wanted from it
    snd_ids = map(rows, layouts) do ids, lay
        g = local_to_global(ids)
        off = 0
        out = Vector{Vector{Int}}()
        for c in lay.recv_counts
            push!(out, Int[g[lay.ghost_lids[off + i]] for i in 1:c])
            off += c
        end
        JaggedArray(out)
    end
    graph = ExchangeGraph(map(lay -> Int.(lay.nbr_ranks) .+ 1, layouts))
    rcv_ids = fetch(exchange(snd_ids, graph))
    # the requests a part received are its send lists (global ids -> own local -> device own)
    map(ctxs, rows, layouts, rcv_ids, graph.rcv) do ctx, ids, lay, req, senders
        g2l = global_to_local(ids)
        send_idx = Int64[]
        send_counts = Int64[]
        for k in 1:length(senders)
            lst = req[k]
            push!(send_counts, length(lst))
            for gid in lst
                push!(send_idx, lay.lid_to_device[g2l[gid]])  # own entries: device own index (1-based)
            end
        end
        # the plan's neighbour order is the receive order; sends go to the same ranks
        @assert Int.(lay.nbr_ranks) .+ 1 == collect(senders) "asymmetric ghost graph"
        ExchangePlan(ctx, lay.n_own, sum(lay.recv_counts; init = 0), lay.nbr_ranks, lay.recv_counts,
                     send_counts, send_idx)
    end
end

# ------------------------------------------------------------------ distributed wrappers
struct HIPPVector{A,B,C}
    parts::A     # DeviceVector per part
    layouts::B   # DeviceLayout per part
    plans::C     # ExchangePlan per part
end
struct HIPPSparseMatrix{A,B,C}
    parts::A     # DeviceMatrix per part
    col_layouts::B
    plans::C
end

"Upload a PVector (own values; ghosts come with the next consistent!)."
function PamgHIP.hip(ctxs, x::PVector; plans = nothing)
    rows = partition(axes(x, 1))
    layouts = map(device_layout, rows)
    plans = plans === nothing ? exchange_plans(ctxs, rows, layouts) : plans
    dv = map(ctxs, partition(x), layouts) do ctx, vals, lay
        PamgHIP.DeviceVector(ctx, vals[lay.own_lids], sum(lay.recv_counts; init = 0))
    end
    HIPPVector(dv, layouts, plans)
end

"Upload a PSparseMatrix: own rows, columns renumbered into the device column layout."
function PamgHIP.hip(ctxs, A::PSparseMatrix)
    rows = partition(axes(A, 1))
    cols = partition(axes(A, 2))
    clay = map(device_layout, cols)
    plans = exchange_plans(ctxs, cols, clay)
    dm = map(ctxs, partition(A), rows, cols, clay, plans) do ctx, Aloc, rids, cids, lay, plan
        # CSR of the own rows (PartitionedArrays local matrices are SparseMatrixCSC over local ids)
        At = sparse(transpose(Aloc[own_to_local(rids), :]))     # column j = own row j
        cg = local_to_global(cids)
        rowptr = Vector{Int64}(At.colptr)
        colv = Vector{Int64}(undef, nnz(At))
        valv = Vector{Float64}(undef, nnz(At))
        for j in 1:size(At, 2)
            rng = At.colptr[j]:(At.colptr[j+1]-1)
            # SPEC §S1: each row in ascending GLOBAL column order
            o = sortperm(cg[At.rowval[rng]])
            colv[rng] = lay.lid_to_device[At.rowval[rng][o]]
            valv[rng] = At.nzval[rng][o]
        end
        PamgHIP.DeviceMatrix(ctx, rowptr, colv, valv, lay.n_own + sum(lay.recv_counts; init = 0);
                             plan = isempty(lay.nbr_ranks) ? nothing : plan, index_base = 1)
    end
    HIPPSparseMatrix(dm, clay, plans)
end

"Own values back into the PartitionedArrays vector."
function Base.copyto!(x::PVector, xd::HIPPVector)
    map(partition(x), xd.parts, xd.layouts) do vals, dv, lay
        vals[lay.own_lids] .= own_values(dv)
    end
    x
end

Base.similar(x::HIPPVector) = HIPPVector(map(similar, x.parts), x.layouts, x.plans)

LinearAlgebra.mul!(y::HIPPVector, A::HIPPSparseMatrix, x::HIPPVector) =
    (foreach(mul!, y.parts, A.parts, x.parts); y)

"consistent!(x): one exchange task per part; `wait` on the result joins them all."
function PamgHIP.consistent!(x::HIPPVector)
    tasks = map(consistent!, x.parts, x.plans)
    PartitionedArrays.Future(() -> (foreach(wait, tasks); x))
end

# Reductions: with an RCCL communicator every part's pamg_vec_dot already returns the global
# sum (all-reduce inside libpamg); without one (debug backend, parts in one process) the part
# sums are added here.
function _global(ctxs, vals)
    r, n = PamgHIP.comm_rank(first(ctxs))
    n > 1 ? first(vals) : sum(vals)
end
LinearAlgebra.dot(x::HIPPVector, y::HIPPVector) =
    _global(map(p -> p.ctx, x.parts), collect(map(dot, x.parts, y.parts)))
LinearAlgebra.norm(x::HIPPVector) = sqrt(dot(x, x))
LinearAlgebra.axpy!(a::Real, x::HIPPVector, y::HIPPVector) = (foreach((xp, yp) -> axpy!(a, xp, yp), x.parts, y.parts); y)
LinearAlgebra.axpby!(a::Real, x::HIPPVector, b::Real, y::HIPPVector) =
    (foreach((xp, yp) -> axpby!(a, xp, b, yp), x.parts, y.parts); y)
Base.fill!(x::HIPPVector, v::Real) = (foreach(p -> fill!(p, v), x.parts); x)
Base.copy!(d::HIPPVector, s::HIPPVector) = (foreach(copy!, d.parts, s.parts); d)

# The V-cycle preconditioner of a distributed hierarchy: one VCycle per part (built by the
# caller from per-part levels; pamg_hier_create with rep_level / rep_offsets).
struct HIPPVCycle{A}
    parts::A
end
LinearAlgebra.ldiv!(x::HIPPVector, M::HIPPVCycle, b::HIPPVector) =
    (foreach(ldiv!, x.parts, M.parts, b.parts); x)

end # module
