/**
 * @file TimeVaryingDCMPlanner.h
 * Batched receding-horizon DCM planner (TimeVaryingDCMPlanner, absent from the reference
 * snapshot), exposed through the reference's Advanceable surface
 * (src/System/include/BipedalLocomotion/System/Advanceable.h:24-46).
 *
 * setContactPhaseLists() stores the plans; the next advance() builds their phase table once: for
 * every phase of every problem the corners pose * (+-L/2, +-W/2, 0) of its active contacts (the
 * rectangle convention of ContinuousContactModel.h:32-36) and their centroid, uploaded, and the
 * phases' support-polygon H-reps built on the device (blf_hull2d_hrep).  It stays resident.
 *
 * Each advance() then runs on the device only (stream-ordered, no host round trip):
 *   1. blf_dcm_phase_expand: knot k of the window, t_k = (start + k) dt, takes the H-rep and
 *      the centroid (r_ref_k = xi_ref_k) of the phase with begin <= t_k < end;
 *   2. blf_dcm_mpc_solve_warm: all QPs, warm-started (after the first advance) from the previous
 *      solution shifted by one knot;
 *   3. the planned xi_1 becomes the next initial DCM (device-to-device copy), the window moves
 *      one knot forward.
 * get() / isValid() download the plan lazily, on the first call after an advance().
 * isValid() is true iff a plan exists and every problem's status is BLF_QP_SOLVED.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_TIME_VARYING_DCM_PLANNER_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_TIME_VARYING_DCM_PLANNER_H

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>
#include <BipedalLocomotion/Planners/ContactPhaseList.h>
#include <BipedalLocomotion/System/Advanceable.h>
#include <BipedalLocomotion/System/VariablesHandler.h>
#include <blf/device.h>

namespace BipedalLocomotion
{
namespace Planners
{

struct DCMPlanBatch
{
    int batch{0};
    int horizon{0};
    double initialTime{0.0};
    std::vector<double> dcm;          /**< [batch][horizon+1][2] */
    std::vector<double> vrp;          /**< [batch][horizon][2]   */
    std::vector<int32_t> status;      /**< [batch] BLF_QP_*      */
    std::vector<int32_t> iterations;  /**< [batch] interior point iterations */
    /** [batch] active-set passes the solve ran (blf_dcm_mpc_solution.passes): what a warm start
     * saves over a cold one */
    std::vector<int32_t> passes;
    /** [batch][n] each problem's QP variables in the planner's VariablesHandler layout
     * (TimeVaryingDCMPlanner::variablesHandler(): "dcm" then "vrp", n = 4 horizon + 2). */
    std::vector<double> variables;
};

class TimeVaryingDCMPlanner : public System::Advanceable<DCMPlanBatch>
{
    blf_dcm_mpc_params m_params{};
    double m_gravity{9.81};
    double m_footLength{0.12};
    double m_footWidth{0.09};
    bool m_warmStart{true};
    double m_warmFloor{1e-3};
    int m_start{0};
    std::vector<ContactPhaseList> m_plans;
    std::vector<double> m_xi0;       /**< [batch][2] */
    std::vector<double> m_height;    /**< [batch][horizon] CoM height per knot (empty: 0.53) */

    // host view of the phase table: the span each problem's window must stay in
    int m_maxPhases{0};
    std::vector<double> m_planBegin, m_planEnd;   /**< [batch] first begin, last end */
    /** [batch] the [begin, end) of every phase without an active contact */
    std::vector<std::vector<std::pair<double, double>>> m_unsupported;
    System::VariablesHandler m_variables;         /**< the QP layout: "dcm", "vrp" */

    bool m_tableDirty{true}, m_omegaDirty{true}, m_xi0Dirty{true};
    bool m_haveWarm{false};
    int m_cur{0};   /**< which of the ping-pong solution buffers holds the latest solve */
    bool m_solved{false};

    // lazily downloaded plan
    mutable bool m_outputDirty{false};
    mutable bool m_valid{false};
    mutable DCMPlanBatch m_output;

    // device-resident state
    blf::DeviceBuffer<double> m_dPhBegin, m_dPhEnd, m_dPhCorners, m_dPhRef, m_dPhA, m_dPhB;
    blf::DeviceBuffer<int32_t> m_dNPhases, m_dPhNCorners, m_dPhNf;
    blf::DeviceBuffer<double> m_dXi0, m_dOmega, m_dXiRef, m_dVrpRef, m_dA, m_dB, m_dWinOmega;
    blf::DeviceBuffer<double> m_dXi, m_dVrp[2], m_dLam[2];
    blf::DeviceBuffer<int32_t> m_dNf, m_dIters, m_dPasses;
    blf::DeviceBuffer<int32_t> m_dStatus[2];   // ping-pong with m_dVrp / m_dLam: the previous
                                                // window's statuses are the next warm start's
                                                // prev_status (a failed problem restarts cold)

    bool buildPhaseTable(blf_handle* h);
    bool checkWindow() const;
    void download() const;

public:
    TimeVaryingDCMPlanner();

    /**
     * Keys (all optional): "horizon" (int), "sampling_time", "gravity", "foot_length",
     * "foot_width", "dcm_weight", "vrp_weight", "terminal_weight" (scalar or 2-vector),
     * "tolerance" (tol_mu), "polish_tolerance" (tol_polish, default 1e-4 for the warm-started windows; 0: interior point
     * only), "max_iterations" (int), "warm_start" (bool, default true), "warm_start_floor"
     * (default 1e-3).
     */
    bool initialize(std::weak_ptr<ParametersHandler::IParametersHandler> handler);

    /** One footstep plan per problem (the batch size). */
    bool setContactPhaseLists(const std::vector<ContactPhaseList>& plans);
    /** Initial DCM per problem ([batch][2]); otherwise each advance() starts at the previous
     * plan's xi_1. */
    bool setInitialDCM(const std::vector<std::array<double, 2>>& xi0);
    /** CoM height per problem and knot ([batch][horizon]); omega_k = sqrt(g / z_k). */
    bool setCoMHeights(const std::vector<double>& heights);

    const DCMPlanBatch& get() const final;
    bool isValid() const final;
    /** Expand the window, solve every problem's QP (warm-started) and move the window one knot.
     * True when the solve was enqueued: a problem whose QP ended at the iteration cap still
     * hands its iterate (xi_1, multipliers) to the next window's warm start; isValid() tells
     * whether every problem of the current plan is solved (status BLF_QP_SOLVED). */
    bool advance() final;

    /** The QP's variable layout (System/src/VariablesHandler.cpp:13-48):
     * "dcm" -> (0, 2 (N + 1)) and "vrp" -> (2 (N + 1), 2 N), registered by initialize(); the
     * plan's `variables` rows are laid out by it. */
    const System::VariablesHandler& variablesHandler() const { return m_variables; }
    const blf_dcm_mpc_params& parameters() const { return m_params; }
    int currentKnot() const { return m_start; }
    /** Device pointers of the latest plan (valid until the next advance() or destruction). */
    blf_dcm_mpc_solution deviceSolution();
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
