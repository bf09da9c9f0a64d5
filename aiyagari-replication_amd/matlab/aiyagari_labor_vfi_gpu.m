% aiyagari_labor_vfi_gpu.m -- host script for the MI355X solver (SURVEY.md §8(b) B6), the
% endogenous-labour VFI model of Aiyagari_Endogenous_Labor_VFI.m.
%
% Calibration, bisection and reporting stay in MATLAB/Octave; the script's two inner loops are one
% gateway call each:
%   * the VFI loop over (a', l) (Aiyagari_Endogenous_Labor_VFI.m:64-122, GE copy :171-228)
%                                                                 -> aiy_labor_vfi_solve_mex
%   * the Monte-Carlo capital path (:127-153, GE copy :231-243)  -> aiy_sim_capital_mex
% The labour, consumption and income paths (:143-147) are interpolated here from the capital and
% state paths the gateway returns, as the script does inside its loop.
% Build the gateways first (aiyagari-replication_amd/mex/Makefile header, or
%   mex -I../../include -L.. -laiyagari_hip <gateway>.c   /   mkoctfile --mex ...).

clear; clc;

% ---------------------------------------------------------------- calibration (:6-62)
beta = 0.96; sigma = 5; alpha = 0.36; delta = 0.08; b = 0;
rho = 0.6; sigma_e = 0.2; N = 7; psi = 1; eta = 2;
Na = 400; tol = 1e-5; max_iter = 1000; T = 10000;
use_step_gateways = false;   % true: keep the script's own VFI loop, one gateway call per sweep

l_grid = ((1:N) - 4) * sigma_e;
edges = [-Inf, ((1:N-1) - 3.5) * sigma_e, Inf];
sd = sigma_e * sqrt(1 - rho^2);
P = zeros(N, N);
for i = 1:N
    for j = 1:N
        P(i, j) = integral(@(x) normpdf(x, rho * l_grid(i), sd), edges(j), edges(j + 1));
    end
end
A = [P' - eye(N); ones(1, N)];
pi_stat = A \ [zeros(N, 1); 1];
s = exp(l_grid);
labor = s * pi_stat;

wmin = (1 - alpha) * (alpha / ((1 / beta - 1) + delta))^(alpha / (1 - alpha));
amin = min(b, wmin * s(1));
kmax = delta^(1 / (alpha - 1));
amax = kmax^alpha + (1 - delta) * kmax;
a_grid = amin + (amax - amin) * linspace(0, 1, Na).^2;
labor_choice = linspace(0.01, 1.5, 10);   % :62

wage = @(r) (1 - alpha) * (alpha / (r + delta))^(alpha / (1 - alpha));
kdemand = @(r) labor * (alpha / (r + delta))^(1 / (1 - alpha));

% ---------------------------------------------------------------- initial solve at r = 0.04
% The script's workspace arrays persist across solves: states with no feasible (a', l) keep
% the previous solve's v_new and policies (:85), so they are passed back in every call.
v_old = zeros(N, Na); v_new = zeros(N, Na);
policy_k = zeros(N, Na); policy_l = zeros(N, Na); policy_c = zeros(N, Na);
r = 0.04;
tic;
if use_step_gateways
    % the reference's loop (:64-122) with its sweep (:69-112) swapped for the gateway; the
    % workspace arrays go back in so infeasible states keep their values (:85)
    for iter = 1:max_iter
        [v_new, policy_k, policy_l, policy_c] = aiy_labor_vfi_sweep_mex(v_old, a_grid, s, P, ...
            labor_choice, r, wage(r), beta, sigma, psi, eta, v_new, policy_k, policy_l, policy_c);
        if max(abs(v_new(:) - v_old(:))) < tol
            break;
        end
        v_old = v_new;
    end
else
    [v_new, v_old, policy_k, policy_l, policy_c, iter] = aiy_labor_vfi_solve_mex( ...
        v_old, a_grid, s, P, labor_choice, r, wage(r), beta, sigma, psi, eta, tol, max_iter, ...
        v_new, policy_k, policy_l, policy_c);
end
fprintf('r = %.4f: %d sweeps\n', r, iter);

% the simulation's first state (:135-136), then one rand per step (:139)
z1 = randi(N);
k1 = a_grid(randi(Na));
[K_s, sim_k, sim_z] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 1);
fprintf('K_s = %.6f\n', K_s);

% ---------------------------------------------------------------- bisection on r (:155-256)
r_low = -0.05; r_high = 1 / beta - 1;
max_r_iter = 10; r_tol = 1e-5;
r_history = zeros(max_r_iter, 1); k_supply = zeros(max_r_iter, 1); k_demand = zeros(max_r_iter, 1);
for r_iter = 1:max_r_iter
    r = (r_low + r_high) / 2;
    w = wage(r);                          % :173 (the labour VFI recomputes w with r)
    % warm start: the previous solve's v_old and workspace arrays (the script's loop state)
    [v_new, v_old, policy_k, policy_l, policy_c, iter] = aiy_labor_vfi_solve_mex( ...
        v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta, tol, max_iter, ...
        v_new, policy_k, policy_l, policy_c);
    [K_s, sim_k, sim_z] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 1);
    K_d = kdemand(r);
    r_history(r_iter) = r; k_supply(r_iter) = K_s; k_demand(r_iter) = K_d;
    fprintf('step %2d: r = %.6f, K_s = %.6f, K_d = %.6f (%d sweeps)\n', r_iter, r, K_s, K_d, iter);
    if abs(K_s - K_d) < r_tol
        break;
    elseif K_s > K_d
        r_high = r;
    else
        r_low = r;
    end
end
fprintf('equilibrium r = %.10f after %.3f s\n', r, toc);

% ---------------------------------------------------------------- the script's reporting paths
% sim_l / sim_c / sim_y / sim_s of :143-147 at the last step, from the returned paths
sim_l = zeros(T, 1); sim_c = zeros(T, 1); sim_y = zeros(T, 1); sim_s = zeros(T, 1);
for t = 2:T
    sim_l(t) = interp1(a_grid, policy_l(sim_z(t), :), sim_k(t - 1), 'linear', 'extrap');
    sim_c(t) = interp1(a_grid, policy_c(sim_z(t), :), sim_k(t - 1), 'linear', 'extrap');
    sim_y(t) = r * sim_k(t) + w * s(sim_z(t)) * sim_l(t);
    sim_s(t) = sim_y(t) + delta * sim_k(t) - sim_c(t);
end
sorted_k = sort(sim_k);
lorenz_k = cumsum(sorted_k) / sum(sorted_k);
gini_k = 1 - 2 * trapz((1:T) / T, lorenz_k);
fprintf('Gini coefficient for wealth: %.4f\n', gini_k);
